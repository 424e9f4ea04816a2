// tieorder.cpp -- origPtr of exactly periodic blocks.
//
// DERIVED WORK NOTICE: the exchange model below follows the B* substring sort and the
// tandem-repeat / Larsson-Sadakane rank refinement of the reference's blocksort.c, which is
// divsufsort:
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
// A block T = w^k (w primitive, |w| = p, k >= 2) has k identical copies of every rotation.
// The BWT does not depend on their order, but origPtr does: it is the slot of rotation 0
// among its k copies, and the reference leaves that choice to the exchange sequence of its
// block sort (the cyclic divsufsort of blocksort.c).  The device sort returns the rank of
// rotation 0 among the p distinct rotations of w (`rank0`); this file computes the copy index
// r, so that origPtr = rank0 * k + r.
//
// Analysis (checked against the reference build on every periodic KAT of SURVEY.md 8a and on
// random periodic blocks, tests/test_abi.py):
//  1. The reference places every suffix by induction from the sorted B* suffixes (cyclic
//     types; B* = a B position followed by an A position): a type-B suffix i is placed when
//     i + 1 is met scanning right to left, a type-A suffix when i + 1 is met scanning left to
//     right (blocksort.c:1439-1501).  Copies of one rotation are met in their slot order and
//     land in the same bucket in that order, so induction preserves the order of the copies.
//  2. Rotation 0 is induced, through positions that are not B*, from the first B* position
//     j0 >= 0 (j0 < p); its copies are induced from the copies j0 + t p of that B* suffix.
//     Hence r = the rank of copy 0 of B* suffix j0 among its k copies in the B* order.
//  3. The B* order is fixed by two stages whose tie order is not a function of the text alone:
//     the substring sort of each (c0, c1) bucket (a multikey quicksort / merge sort on the B*
//     substrings, blocksort.c:302-664) and the rank refinement (tr / ls doubling on the
//     reduced string, blocksort.c:669-1309).  Among copies every comparison ties, so the copy
//     order is the product of the element exchanges those stages perform on the whole
//     bucket / reduced string.  There is no closed form (the copy rank moves with k in a
//     pattern set by pivot positions, merge interleaving and the doubling budget), so this
//     file re-enacts the exchanges: only the B* level (m = k * |B* of w| items, not n), and
//     only the permutation of items (no output column).
// The exchange model below is written from that analysis; its elementary operations (median
// pivots, heap sort, 3-way partition, buffered merges, the bucket block driver, the depth
// doubling with its work budget) are shared where the reference duplicates them for its two
// stages, each operating on an abstract key functor.
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "tieorder.h"

namespace bzg {
namespace {

using I32 = int32_t;

// ------------------------------------------------------------------ shared primitives
inline int ilog2_floor(uint32_t v) {  // floor(log2 v), -1 for 0
  return v == 0 ? -1 : 31 - __builtin_clz(v);
}
// the stages' depth limits use lg on 16-bit (substring stage) or 32-bit (rank stage) sizes
inline int lg16(I32 v) { return ilog2_floor((uint32_t)v & 0xffffu); }
inline int lg32(I32 v) { return ilog2_floor((uint32_t)v); }

// Median-of-three / five / nine position chooser over an array `a` with key K(index).
template <typename Key>
struct Pivot {
  I32* a;
  Key K;
  I32 med3(I32 x, I32 y, I32 z) const {
    if (K(a[x]) > K(a[y])) std::swap(x, y);
    if (K(a[y]) > K(a[z])) return K(a[x]) > K(a[z]) ? x : z;
    return y;
  }
  I32 med5(I32 p1, I32 p2, I32 p3, I32 p4, I32 p5) const {
    if (K(a[p2]) > K(a[p3])) std::swap(p2, p3);
    if (K(a[p4]) > K(a[p5])) std::swap(p4, p5);
    if (K(a[p2]) > K(a[p4])) {
      std::swap(p2, p4);
      std::swap(p3, p5);
    }
    if (K(a[p1]) > K(a[p3])) std::swap(p1, p3);
    if (K(a[p1]) > K(a[p4])) {
      std::swap(p1, p4);
      std::swap(p3, p5);
    }
    return K(a[p3]) > K(a[p4]) ? p4 : p3;
  }
  // index of the pivot of [lo, hi)
  I32 choose(I32 lo, I32 hi) const {
    I32 t = hi - lo;
    const I32 mid = lo + t / 2;
    if (t <= 512) {
      if (t <= 32) return med3(lo, mid, hi - 1);
      t >>= 2;
      return med5(lo, lo + t, mid, hi - 1 - t, hi - 1);
    }
    t >>= 3;
    return med3(med3(lo, lo + t, lo + (t << 1)), med3(mid - t, mid, mid + t),
                med3(hi - 1 - (t << 1), hi - 1 - t, hi - 1));
  }
};

// In-place heap sort of a[lo, lo + size) by K (max-heap; an odd heap with the even case's
// extra element merged in first).  The sift reads the right sibling even when it is the
// first slot past the heap, as the reference's sift does.
template <typename Key>
void heap_sort(I32* a, I32 size, const Key& K) {
  auto sift = [&](I32 i, I32 sz) {
    const I32 v = a[i];
    const auto c = K(v);
    I32 j;
    while ((j = 2 * i + 1) < sz) {
      I32 k = j++;
      auto d = K(a[k]);
      const auto e = K(a[j]);
      if (d < e) {
        k = j;
        d = e;
      }
      if (d <= c) break;
      a[i] = a[k];
      i = k;
    }
    a[i] = v;
  };
  I32 m = size;
  if (size % 2 == 0) {
    m--;
    if (K(a[m / 2]) < K(a[m])) std::swap(a[m], a[m / 2]);
  }
  for (I32 i = m / 2 - 1; i >= 0; --i) sift(i, m);
  if (size % 2 == 0) {
    std::swap(a[0], a[m]);
    sift(0, m);
  }
  for (I32 i = m - 1; i > 0; --i) {
    const I32 t = a[0];
    a[0] = a[i];
    sift(0, i);
    a[i] = t;
  }
}

// Three-way split of a[lo, hi) around value v: afterwards [lo, lt) < v, [lt, gt) == v,
// [gt, hi) > v.  `scan` is where the forward scan starts (lo + 1 when a[lo] is the pivot
// itself, lo otherwise).  Returns false (nothing moved) when every element equals v.  The
// equal elements are first collected at both ends during the scan and then swapped into the
// middle, which fixes the order the equal elements (the ties) end in.
template <typename Key>
bool split3(I32* a, I32 lo, I32 hi, I32 scan, I32 v, const Key& K, I32& lt, I32& gt) {
  I32 b = scan - 1, x = 0;
  while (++b < hi && (x = K(a[b])) == v) {
  }
  I32 el = b;  // end of the equal run collected at the front
  if (b < hi && x < v) {
    while (++b < hi && (x = K(a[b])) <= v)
      if (x == v) std::swap(a[b], a[el++]);
  }
  I32 c = hi;
  while (b < --c && (x = K(a[c])) == v) {
  }
  I32 er = c;  // start of the equal run collected at the back (inclusive)
  if (b < er && x > v) {
    while (b < --c && (x = K(a[c])) >= v)
      if (x == v) std::swap(a[c], a[er--]);
  }
  while (b < c) {
    std::swap(a[b], a[c]);
    while (++b < c && (x = K(a[b])) <= v)
      if (x == v) std::swap(a[b], a[el++]);
    while (b < --c && (x = K(a[c])) >= v)
      if (x == v) std::swap(a[c], a[er--]);
  }
  if (el > er) return false;
  const I32 last_lt = b - 1;
  I32 s = std::min(el - lo, b - el);
  for (I32 e = lo, f = b - s; s > 0; --s, ++e, ++f) std::swap(a[e], a[f]);
  s = std::min(er - last_lt, hi - er - 1);
  for (I32 e = b, f = hi - s; s > 0; --s, ++e, ++f) std::swap(a[e], a[f]);
  lt = lo + (b - el);
  gt = hi - (er - last_lt);
  return true;
}

// ------------------------------------------------------------------ the B* level
// Cyclic text with the reference's two guard characters (T[-1] = T[n-1], T[n] = T[0]).
struct Text {
  std::vector<uint8_t> buf;
  I32 n = 0;
  void set(const uint8_t* t, I32 len) {
    n = len;
    buf.assign((size_t)len + 8, 0);
    std::memcpy(buf.data() + 1, t, (size_t)len);
    buf[0] = t[len - 1];
    buf[(size_t)len + 1] = t[0];
  }
  int at(I32 i) const { return buf[(size_t)(i + 1)]; }  // -1 <= i <= n + 6
};

// ------------------------------------------------------------------ stage 1: substrings
// Items are B* indices j (PA[j] = text position, ascending).  The key of item j at depth d
// is character PA[j] + 2 + d; item j's substring ends at character PA[j + 1] + 2 (the next B*
// position plus two).  Negative entries (~j) mark an item equal to the item before it.
class SubstringStage {
 public:
  SubstringStage(const Text& T, const I32* PA, I32 m, I32 n) : T_(T), PA_(PA), m_(m), n_(n) {}

  // Sorts the bucket a[lo, hi) using buf[0, bufsize) as merge scratch (last: the bucket starts
  // with the item m - 1, whose substring wraps around the text end).
  void sort_bucket(I32* a, I32 lo, I32 hi, I32* buf, I32 bufsize, bool last) {
    constexpr I32 kBlock = 1024;
    if (last) ++lo;
    I32 s = lo, i = 0;
    for (; s + kBlock < hi; s += kBlock, ++i) {
      multikey(a, s, s + kBlock);
      I32* cur = a + s + kBlock;
      I32 cursize = hi - (s + kBlock);
      if (cursize <= bufsize) {
        cursize = bufsize;
        cur = buf;
      }
      for (I32 b = s, k = kBlock, j = i; j & 1; b -= k, k <<= 1, j >>= 1) merge(a, b - k, b, b + k, cur, cursize);
    }
    multikey(a, s, hi);
    for (I32 k = kBlock; i != 0; k <<= 1, i >>= 1)
      if (i & 1) {
        merge(a, s - k, s, hi, buf, bufsize);
        s -= k;
      }
    if (last) insert_wrapping(a, lo, hi);
  }

 private:
  int key(I32 item, I32 d) const { return T_.at(PA_[item] + 2 + d); }
  int before(I32 item, I32 d) const { return T_.at(PA_[item] + 2 + d - 1); }
  bool ended(I32 item, I32 d) const { return PA_[item] + d >= PA_[item + 1] - 1; }

  // compare the substrings of items x and y from depth d (both end at their next B* + 2)
  int cmp(I32 x, I32 y, I32 d) const {
    I32 u = PA_[x] + 2 + d, v = PA_[y] + 2 + d;
    const I32 ue = PA_[x + 1] + 2, ve = PA_[y + 1] + 2;
    while (u < ue && v < ve && T_.at(u) == T_.at(v)) {
      ++u;
      ++v;
    }
    if (u < ue) return v < ve ? T_.at(u) - T_.at(v) : 1;
    return v < ve ? -1 : 0;
  }

  // the wrapping item m - 1 against item y (its substring runs to the text end, then on from
  // position 2 to the first B* position + 2)
  int cmp_wrap(I32 y) const {
    I32 u = PA_[m_ - 1] + 2, v = PA_[y] + 2;
    const I32 ve = PA_[y + 1] + 2;
    I32 ue = n_;
    while (u < ue && v < ve && T_.at(u) == T_.at(v)) {
      ++u;
      ++v;
    }
    if (u < ue) return v < ve ? T_.at(u) - T_.at(v) : 1;
    if (v == ve) return 1;
    u -= n_;
    ue = PA_[0] + 2;
    while (u < ue && v < ve && T_.at(u) == T_.at(v)) {
      ++u;
      ++v;
    }
    if (u < ue) return v < ve ? T_.at(u) - T_.at(v) : 1;
    return v < ve ? -1 : 0;
  }

  // items of a[lo, hi) whose substring ends at depth d to the front (marked), the rest after;
  // returns the first of the rest
  I32 split_ended(I32* a, I32 lo, I32 hi, I32 d) const {
    I32 x = lo - 1, y = hi;
    for (;;) {
      while (++x < y && ended(a[x], d)) a[x] = ~a[x];
      while (x < --y && !ended(a[y], d)) {
      }
      if (y <= x) break;
      const I32 t = ~a[y];
      a[y] = a[x];
      a[x] = t;
    }
    if (lo < x) a[lo] = ~a[lo];
    return x;
  }

  // insertion sort of a[lo, hi) from depth d, right to left; equal neighbours are marked
  void insertion(I32* a, I32 lo, I32 hi, I32 d) const {
    for (I32 i = hi - 2; lo <= i; --i) {
      const I32 t = a[i];
      I32 j = i + 1, r;
      while ((r = cmp(t, a[j], d)) > 0) {
        do {
          a[j - 1] = a[j];
        } while (++j < hi && a[j] < 0);
        if (hi <= j) break;
      }
      if (r == 0) a[j] = ~a[j];
      a[j - 1] = t;
    }
  }

  // multikey quicksort of a[lo, hi) (introsort: heap sort once the depth budget is spent)
  void multikey(I32* a, I32 lo, I32 hi) const {
    struct Frame {
      I32 lo, hi, d, limit;
    };
    std::vector<Frame> st;
    I32 d = 0, limit = lg16(hi - lo);
    auto pop = [&]() {
      if (st.empty()) return false;
      const Frame f = st.back();
      st.pop_back();
      lo = f.lo;
      hi = f.hi;
      d = f.d;
      limit = f.limit;
      return true;
    };
    for (;;) {
      if (hi - lo <= 8) {
        if (hi - lo > 1) insertion(a, lo, hi, d);
        if (!pop()) return;
        continue;
      }
      const auto K = [&](I32 item) { return key(item, d); };
      if (limit-- == 0) heap_sort(a + lo, hi - lo, K);
      if (limit < 0) {  // keys in order: peel the first run of equal keys
        I32 e = lo + 1;
        int v = key(a[lo], d);
        for (; e < hi; ++e) {
          const int x = key(a[e], d);
          if (x != v) {
            if (e - lo > 1) break;
            v = x;
            lo = e;
          }
        }
        if (before(a[lo], d) < v) lo = split_ended(a, lo, e, d);
        if (e - lo <= hi - e) {
          if (e - lo > 1) {
            st.push_back({e, hi, d, -1});
            hi = e;
            d += 1;
            limit = lg16(e - lo);
          } else {
            lo = e;
            limit = -1;
          }
        } else {
          if (hi - e > 1) {
            st.push_back({lo, e, d + 1, lg16(e - lo)});
            lo = e;
            limit = -1;
          } else {
            hi = e;
            d += 1;
            limit = lg16(e - lo);
          }
        }
        continue;
      }
      const Pivot<decltype(K)> pv{a, K};
      const I32 p = pv.choose(lo, hi);
      const int v = key(a[p], d);
      std::swap(a[lo], a[p]);
      I32 lt, gt;
      if (split3(a, lo, hi, lo + 1, v, K, lt, gt)) {
        // [lt, gt) share this character: their substrings continue one deeper, except those
        // that end here (moved to its front)
        const I32 mid = v <= before(a[lt], d) ? lt : split_ended(a, lt, gt, d);
        const I32 nl = lt - lo, nr = hi - gt, ne = gt - mid;
        if (nl <= nr) {
          if (nr <= ne) {
            st.push_back({mid, gt, d + 1, lg16(ne)});
            st.push_back({gt, hi, d, limit});
            hi = lt;
          } else if (nl <= ne) {
            st.push_back({gt, hi, d, limit});
            st.push_back({mid, gt, d + 1, lg16(ne)});
            hi = lt;
          } else {
            st.push_back({gt, hi, d, limit});
            st.push_back({lo, lt, d, limit});
            lo = mid;
            hi = gt;
            d += 1;
            limit = lg16(ne);
          }
        } else {
          if (nl <= ne) {
            st.push_back({mid, gt, d + 1, lg16(ne)});
            st.push_back({lo, lt, d, limit});
            lo = gt;
          } else if (nr <= ne) {
            st.push_back({lo, lt, d, limit});
            st.push_back({mid, gt, d + 1, lg16(ne)});
            lo = gt;
          } else {
            st.push_back({lo, lt, d, limit});
            st.push_back({gt, hi, d, limit});
            lo = mid;
            hi = gt;
            d += 1;
            limit = lg16(ne);
          }
        }
      } else {  // one character everywhere: go one deeper
        limit += 1;
        if (before(a[lo], d) < v) {
          lo = split_ended(a, lo, hi, d);
          limit = lg16(hi - lo);
        }
        d += 1;
      }
    }
  }

  // ---- merging two sorted runs (substrings compared from depth 0)
  static I32 idx(I32 x) { return x >= 0 ? x : ~x; }
  int cmp0(I32 x, I32 y) const { return cmp(x, y, 0); }
  static void swap_blocks(I32* p, I32* q, I32 size) {
    for (I32 i = 0; i < size; ++i) std::swap(p[i], q[i]);
  }

  // [lo, mid) through the buffer (the shorter, left run)
  void merge_front(I32* a, I32* buf, I32 lo, I32 mid, I32 hi) const {
    I32* bufend = buf + (mid - lo);
    swap_blocks(buf, a + lo, mid - lo);
    I32* i = a + lo;
    I32* j = buf;
    I32* k = a + mid;
    I32* end = a + hi;
    const I32 t = a[lo];
    auto from_j = [&]() {
      *i++ = *j;
      *j++ = *i;
    };
    auto from_k = [&]() {
      *i++ = *k;
      *k++ = *i;
    };
    for (;;) {
      const int r = cmp0(*j, *k);
      if (r < 0) {
        do {
          from_j();
          if (bufend <= j) {
            *(bufend - 1) = t;
            return;
          }
        } while (*j < 0);
      } else if (r > 0) {
        do {
          from_k();
          if (end <= k) {
            do from_j();
            while (j < bufend);
            *(bufend - 1) = t;
            return;
          }
        } while (*k < 0);
      } else {
        *k = ~*k;
        do {
          from_j();
          if (bufend <= j) {
            *(bufend - 1) = t;
            return;
          }
        } while (*j < 0);
        do {
          from_k();
          if (end <= k) {
            do from_j();
            while (j < bufend);
            *(bufend - 1) = t;
            return;
          }
        } while (*k < 0);
      }
    }
  }

  // [mid, hi) through the buffer, merging from the back
  void merge_back(I32* a, I32* buf, I32 lo, I32 mid, I32 hi) const {
    I32* bufend = buf + (hi - mid);
    swap_blocks(buf, a + mid, hi - mid);
    I32* i = a + hi - 1;
    I32* j = bufend - 1;
    I32* k = a + mid - 1;
    I32* first = a + lo;
    const I32 t = a[hi - 1];
    bool jm = *j < 0, km = *k < 0;  // the current item is a marked (equal) one
    I32 pj = idx(*j), pk = idx(*k);
    auto from_j = [&]() {
      *i-- = *j;
      *j-- = *i;
    };
    auto from_k = [&]() {
      *i-- = *k;
      *k-- = *i;
    };
    for (;;) {
      const int r = cmp0(pj, pk);
      if (r > 0) {
        if (jm) do from_j();
          while (*j < 0);
        from_j();
        if (j < buf) {
          *buf = t;
          return;
        }
        jm = *j < 0;
        pj = idx(*j);
      } else if (r < 0) {
        if (km) do from_k();
          while (*k < 0);
        from_k();
        if (k < first) {
          do from_j();
          while (buf <= j);
          *buf = t;
          return;
        }
        km = *k < 0;
        pk = idx(*k);
      } else {
        if (jm) do from_j();
          while (*j < 0);
        *i-- = ~*j;
        *j-- = *i;
        if (j < buf) {
          *buf = t;
          return;
        }
        if (km) do from_k();
          while (*k < 0);
        from_k();
        if (k < first) {
          while (buf <= j) from_j();
          *buf = t;
          return;
        }
        jm = *j < 0;
        pj = idx(*j);
        km = *k < 0;
        pk = idx(*k);
      }
    }
  }

  // merge of the sorted runs a[lo, mid) and a[mid, hi): through the buffer when a run fits
  // it, otherwise by exchanging the overlapping blocks found by a binary search (a symmetric
  // merge) and recursing on both sides; boundary items are re-checked for equality.
  void merge(I32* a, I32 lo, I32 mid, I32 hi, I32* buf, I32 bufsize) const {
    struct Frame {
      I32 lo, mid, hi, check;
    };
    std::vector<Frame> st;
    I32 check = 0;
    auto mark_if_equal = [&](I32 p) {
      if (a[p] >= 0 && cmp0(idx(a[p - 1]), a[p]) == 0) a[p] = ~a[p];
    };
    auto pop = [&]() {
      if (st.empty()) return false;
      const Frame f = st.back();
      st.pop_back();
      lo = f.lo;
      mid = f.mid;
      hi = f.hi;
      check = f.check;
      return true;
    };
    for (;;) {
      if (hi - mid <= bufsize) {
        if (lo < mid && mid < hi) merge_back(a, buf, lo, mid, hi);
        if (check & 1) mark_if_equal(lo);
        if (check & 2) mark_if_equal(hi);
        if (!pop()) return;
        continue;
      }
      if (mid - lo <= bufsize) {
        if (lo < mid) merge_front(a, buf, lo, mid, hi);
        if (check & 1) mark_if_equal(lo);
        if (check & 2) mark_if_equal(hi);
        if (!pop()) return;
        continue;
      }
      I32 m = 0;
      for (I32 len = std::min(mid - lo, hi - mid), half = len >> 1; len > 0; len = half, half >>= 1) {
        if (cmp0(idx(a[mid + m + half]), idx(a[mid - m - half - 1])) < 0) {
          m += half + 1;
          half -= (len & 1) ^ 1;
        }
      }
      if (m > 0) {
        swap_blocks(a + mid - m, a + mid, m);
        I32 i = mid, j = mid, next = 0;
        if (mid + m < hi) {
          if (a[mid + m] < 0) {
            while (a[i - 1] < 0) --i;
            a[mid + m] = ~a[mid + m];
          }
          for (j = mid; a[j] < 0; ++j) {
          }
          next = 1;
        }
        if (i - lo <= hi - j) {
          st.push_back({j, mid + m, hi, (check & 2) | (next & 1)});
          mid -= m;
          hi = i;
          check &= 1;
        } else {
          if (i == mid && mid == j) next <<= 1;
          st.push_back({lo, mid - m, i, (check & 1) | (next & 2)});
          lo = j;
          mid += m;
          check = (check & 2) | (next & 1);
        }
      } else {
        if (check & 1) mark_if_equal(lo);
        mark_if_equal(mid);
        if (check & 2) mark_if_equal(hi);
        if (!pop()) return;
      }
    }
  }

  // the wrapping item m - 1 (in a[lo - 1]) moves right past the items it is larger than
  void insert_wrapping(I32* a, I32 lo, I32 hi) const {
    const I32 w = a[lo - 1];
    I32 p = lo, r = 1;
    while (p < hi && (a[p] < 0 || (r = cmp_wrap(a[p])) > 0)) {
      a[p - 1] = a[p];
      ++p;
    }
    if (r == 0) a[p] = ~a[p];
    a[p - 1] = w;
  }

  const Text& T_;
  const I32* PA_;
  I32 m_, n_;
};

// ------------------------------------------------------------------ stage 2: rank refinement
// Items are B* indices; R[j] is item j's rank (the last slot of its group); the reduced string
// is cyclic, so the key of item j at offset d is R[(j + d) mod m].  S holds the order: a
// non-negative entry is an item, a negative entry -L at the head of a run says "the next L
// slots are final".  Groups are refined by 3-way quicksort on the key at offset d (d grows by
// one per level, with heap sort past the depth limit, insertion sort for small ranges, and
// the "-1 / -2 / -3 / -4" follow-up states of the level machine); when the work budget is
// spent the rest is finished by plain doubling (offset doubles per round).
class RankStage {
 public:
  RankStage(I32* S, I32* R, I32 m) : S_(S), R_(R), m_(m) {}

  void run(I32 d0) {
    if (S_[0] <= -m_) return;  // every item already final
    I32 budget = (lg32(m_) * 2 / 3 + 1) * m_;
    I32 first = 0;
    do {
      const I32 t = S_[first];
      if (t < 0) {
        first -= t;
      } else {
        const I32 last = R_[t] + 1;
        refine(first, last, d0, budget);
        first = last;
        if (budget <= 0) {
          S_[0] = -first;
          doubling(d0);
          break;
        }
      }
    } while (first < m_);
  }

 private:
  I32 key(I32 item, I32 d) const {  // R at (item + d), cyclic (d < 2m)
    I32 q = item + d;
    if (q >= m_) q -= m_;
    return R_[q];
  }

  void insertion(I32 lo, I32 hi, I32 d) {
    for (I32 a = lo + 1; a < hi; ++a) {
      const I32 t = S_[a];
      I32 b = a - 1, r;
      while ((r = key(t, d) - key(S_[b], d)) < 0) {
        do {
          S_[b + 1] = S_[b];
        } while (lo <= --b && S_[b] < 0);
        if (b < lo) break;
      }
      if (r == 0) S_[b] = ~S_[b];
      S_[b + 1] = t;
    }
  }

  // a run of marked (equal) items starting at `lo` plus its unmarked last item: unmark, give
  // the run its rank when more follows, return one past the run
  I32 take_run(I32 lo, I32 hi) {
    I32 b = lo;
    do S_[b] = ~S_[b];
    while (S_[++b] < 0);
    return b;  // the run's last item
  }
  void rank_range(I32 lo, I32 hi, I32 v) {
    for (I32 c = lo; c < hi; ++c) R_[S_[c]] = v;
  }
  // leading final items (non-negative entries) of [lo, hi): each ranked at its slot
  I32 settle_prefix(I32 lo, I32 hi) {
    if (S_[lo] >= 0) {
      I32 a = lo;
      do R_[S_[a]] = a;
      while (++a < hi && S_[a] >= 0);
      return a;
    }
    return lo;
  }

  void copy_down(I32 lo, I32 a, I32 b, I32 hi, I32 depth) {
    const I32 v = b - 1;
    I32 d = a - 1;
    for (I32 c = lo; c <= d; ++c) {
      I32 s = S_[c] - depth;
      if (s < 0) s += m_;
      if (R_[s] == v) {
        S_[++d] = s;
        R_[s] = d;
      }
    }
    I32 e = d + 1;
    d = b;
    for (I32 c = hi - 1; e < d; --c) {
      I32 s = S_[c] - depth;
      if (s < 0) s += m_;
      if (R_[s] == v) {
        S_[--d] = s;
        R_[s] = d;
      }
    }
  }

  struct Frame {
    I32 d, lo, hi, state;  // d < 0: the (lo, hi) record consumed by a state -2 frame
  };

  void refine(I32 lo, I32 hi, I32 d, I32& budget) {
    std::vector<Frame> st;
    I32 limit = lg32(hi - lo);
    auto pop = [&]() {
      if (st.empty()) return false;
      const Frame f = st.back();
      st.pop_back();
      d = f.d;
      lo = f.lo;
      hi = f.hi;
      limit = f.state;
      return true;
    };
    for (;;) {
      const auto K = [&](I32 item) { return key(item, d); };
      if (limit < 0) {
        if (limit == -1) {  // split by the key one offset back against the group's own rank
          I32 a = lo, b = hi;
          const auto Kb = [&](I32 item) { return key(item, d - 1); };
          split3(S_, lo, hi, lo, hi - 1, Kb, a, b);
          if (lo < a || b < hi) {
            if (a < hi) rank_range(lo, a, a - 1);
            if (b < hi) rank_range(a, b, b - 1);
            if (b - a > 1) {
              st.push_back({-1, a, b, 0});
              st.push_back({d - 1, lo, hi, -2});
            }
            if (a - lo <= hi - b) {
              if (a - lo > 1) {
                st.push_back({d, b, hi, lg32(hi - b)});
                hi = a;
                limit = lg32(a - lo);
              } else if (hi - b > 1) {
                lo = b;
                limit = lg32(hi - b);
              } else if (!pop()) {
                return;
              }
            } else {
              if (hi - b > 1) {
                st.push_back({d, lo, a, lg32(a - lo)});
                lo = b;
                limit = lg32(hi - b);
              } else if (a - lo > 1) {
                hi = a;
                limit = lg32(a - lo);
              } else if (!pop()) {
                return;
              }
            }
          } else {
            for (I32 c = lo; c < hi; ++c) R_[S_[c]] = c;
            if (!pop()) return;
          }
        } else if (limit == -2) {  // ranks of the tied middle from the finished neighbours
          const Frame rec = st.back();
          st.pop_back();
          copy_down(lo, rec.lo, rec.hi, hi, d);
          if (!pop()) return;
        } else {  // -3: the range is sorted; walk its runs
          lo = settle_prefix(lo, hi);
          if (lo < hi) {
            const I32 b = take_run(lo, hi);
            const I32 a = b + 1;
            const I32 next = R_[S_[b]] != key(S_[b], d) ? lg32(a - lo) : -1;
            if (a < hi) rank_range(lo, a, a - 1);
            if (a - lo <= hi - a) {
              st.push_back({d, a, hi, -3});
              d += 1;
              hi = a;
              limit = next;
            } else if (hi - a > 1) {
              st.push_back({d + 1, lo, a, next});
              lo = a;
              limit = -3;
            } else {
              d += 1;
              hi = a;
              limit = next;
            }
          } else if (!pop()) {
            return;
          }
        }
        continue;
      }
      if (hi - lo <= 8) {
        budget -= hi - lo;
        insertion(lo, hi, d);
        for (;;) {
          lo = settle_prefix(lo, hi);
          if (lo < hi) {
            const I32 b = take_run(lo, hi);
            const I32 a = b + 1;
            if (R_[S_[b]] == key(S_[b], d)) limit = -1;
            if (a < hi) rank_range(lo, a, a - 1);
            if (hi - a > 1) st.push_back({d, a, hi, -4});
            d += 1;
            hi = a;
            if (limit == -1) break;
            budget -= hi - lo;
            insertion(lo, hi, d);
          } else {
            if (!pop()) return;
            if (limit != -4) break;
          }
        }
        continue;
      }
      if (limit-- == 0) {
        budget -= hi - lo;
        heap_sort(S_ + lo, hi - lo, K);
        I32 v = key(S_[hi - 1], d);
        for (I32 a = hi - 2; lo <= a; --a) {
          const I32 x = key(S_[a], d);
          if (x == v) S_[a] = ~S_[a];
          else v = x;
        }
        limit = -3;
        continue;
      }
      const Pivot<decltype(K)> pv{S_, K};
      const I32 p = pv.choose(lo, hi);
      std::swap(S_[lo], S_[p]);
      const I32 v = key(S_[lo], d);
      I32 a, b;
      if (split3(S_, lo, hi, lo + 1, v, K, a, b)) {
        const I32 next = R_[S_[a]] == key(S_[a], d) ? -1 : lg32(b - a);
        rank_range(lo, a, a - 1);
        if (b < hi) rank_range(a, b, b - 1);
        budget -= hi - lo;
        const I32 nl = a - lo, nr = hi - b, ne = b - a;
        if (nl <= nr) {
          if (nr <= ne) {
            if (nl > 1) {
              st.push_back({d + 1, a, b, next});
              st.push_back({d, b, hi, limit});
              hi = a;
            } else if (nr > 1) {
              st.push_back({d + 1, a, b, next});
              lo = b;
            } else if (ne > 1) {
              d += 1;
              lo = a;
              hi = b;
              limit = next;
            } else if (!pop()) {
              return;
            }
          } else if (nl <= ne) {
            if (nl > 1) {
              st.push_back({d, b, hi, limit});
              st.push_back({d + 1, a, b, next});
              hi = a;
            } else if (ne > 1) {
              st.push_back({d, b, hi, limit});
              d += 1;
              lo = a;
              hi = b;
              limit = next;
            } else {
              lo = b;
            }
          } else {
            if (ne > 1) {
              st.push_back({d, b, hi, limit});
              st.push_back({d, lo, a, limit});
              d += 1;
              lo = a;
              hi = b;
              limit = next;
            } else {
              st.push_back({d, b, hi, limit});
              hi = a;
            }
          }
        } else {
          if (nl <= ne) {
            if (nr > 1) {
              st.push_back({d + 1, a, b, next});
              st.push_back({d, lo, a, limit});
              lo = b;
            } else if (nl > 1) {
              st.push_back({d + 1, a, b, next});
              hi = a;
            } else if (ne > 1) {
              d += 1;
              lo = a;
              hi = b;
              limit = next;
            } else if (!pop()) {
              return;
            }
          } else if (nr <= ne) {
            if (nr > 1) {
              st.push_back({d, lo, a, limit});
              st.push_back({d + 1, a, b, next});
              lo = b;
            } else if (ne > 1) {
              st.push_back({d, lo, a, limit});
              d += 1;
              lo = a;
              hi = b;
              limit = next;
            } else {
              hi = a;
            }
          } else {
            if (ne > 1) {
              st.push_back({d, lo, a, limit});
              st.push_back({d, b, hi, limit});
              d += 1;
              lo = a;
              hi = b;
              limit = next;
            } else {
              st.push_back({d, lo, a, limit});
              lo = b;
            }
          }
        }
      } else {  // one key everywhere: one offset deeper (or done when it is the group itself)
        limit = R_[S_[lo]] == key(S_[lo], d) ? -1 : limit + 1;
        d += 1;
        budget -= hi - lo;
      }
    }
  }

  // ---- doubling: every unfinished group sorted on the key at offset d, then d doubles
  void group_ranks(I32 lo, I32 hi) {
    for (I32 a = lo; a < hi; ++a) {
      if (S_[a] >= 0) {
        const I32 b = a;
        do R_[S_[a]] = a;
        while (++a < hi && S_[a] >= 0);
        S_[b] = b - a;
        if (hi <= a) break;
      }
      const I32 b = a;
      do S_[a] = ~S_[a];
      while (S_[++a] < 0);
      for (I32 c = b; c <= a; ++c) R_[S_[c]] = a;
    }
  }

  void sort_level(I32 lo, I32 hi, I32 d) {
    struct F3 {
      I32 lo, hi, limit;
    };
    std::vector<F3> st;
    I32 limit = lg32(hi - lo);
    const auto K = [&](I32 item) { return key(item, d); };
    auto pop = [&]() {
      if (st.empty()) return false;
      const F3 f = st.back();
      st.pop_back();
      lo = f.lo;
      hi = f.hi;
      limit = f.limit;
      return true;
    };
    for (;;) {
      if (hi - lo <= 8) {
        if (hi - lo > 1) {
          insertion(lo, hi, d);
          group_ranks(lo, hi);
        } else if (hi - lo == 1) {
          S_[lo] = -1;
        }
        if (!pop()) return;
        continue;
      }
      if (limit-- == 0) {
        heap_sort(S_ + lo, hi - lo, K);
        I32 v = key(S_[hi - 1], d);
        for (I32 a = hi - 2; lo <= a; --a) {
          const I32 x = key(S_[a], d);
          if (x == v) S_[a] = ~S_[a];
          else v = x;
        }
        group_ranks(lo, hi);
        if (!pop()) return;
        continue;
      }
      const Pivot<decltype(K)> pv{S_, K};
      const I32 p = pv.choose(lo, hi);
      std::swap(S_[lo], S_[p]);
      const I32 v = key(S_[lo], d);
      I32 a, b;
      if (split3(S_, lo, hi, lo + 1, v, K, a, b)) {
        rank_range(lo, a, a - 1);
        if (b < hi) rank_range(a, b, b - 1);
        if (b - a == 1) S_[a] = -1;
        if (a - lo <= hi - b) {
          if (lo < a) {
            st.push_back({b, hi, limit});
            hi = a;
          } else {
            lo = b;
          }
        } else {
          if (b < hi) {
            st.push_back({lo, a, limit});
            lo = b;
          } else {
            hi = a;
          }
        }
      } else if (!pop()) {
        return;
      }
    }
  }

  void doubling(I32 d) {
    for (; S_[0] > -m_; d += d) {
      I32 first = 0, skip = 0;
      do {
        const I32 t = S_[first];
        if (t < 0) {
          first -= t;
          skip += t;
        } else {
          if (skip != 0) {
            S_[first + skip] = skip;
            skip = 0;
          }
          const I32 last = R_[t] + 1;
          sort_level(first, last, d);
          first = last;
        }
      } while (first < m_);
      if (skip != 0) S_[first + skip] = skip;
      if (m_ < d) {  // past the string length: the remaining ties are final in slot order
        first = 0;
        do {
          const I32 t = S_[first];
          if (t < 0) {
            first -= t;
          } else {
            const I32 last = R_[t] + 1;
            for (I32 i = first; i < last; ++i) R_[S_[i]] = i;
            first = last;
          }
        } while (first < m_);
        break;
      }
    }
  }

  I32* S_;
  I32* R_;
  I32 m_;
};

// ------------------------------------------------------------------ driver
// Copy index r of rotation 0 of the periodic block t[0, n) with primitive period p.
I32 copy_rank(const uint8_t* t, I32 n, I32 p) {
  Text T;
  T.set(t, n);
  // cyclic types: B = smaller than the next rotation; B* = B followed by A
  std::vector<uint8_t> isB(n);
  {
    I32 i0 = -1;  // a position whose type is decided by a strict comparison
    for (I32 i = 0; i < n; i++)
      if (t[i] != t[(i + 1) % n]) {
        i0 = i;
        break;
      }
    if (i0 < 0) return 0;  // one symbol: no B* suffix (blocksort.c:1349)
    isB[i0] = t[i0] < t[(i0 + 1) % n];
    for (I32 s = 1; s < n; s++) {  // walk backwards from i0
      const I32 i = (i0 - s + n) % n, nx = (i + 1) % n;
      isB[i] = t[i] < t[nx] || (t[i] == t[nx] && isB[nx]);
    }
  }
  std::vector<I32> PA;
  for (I32 i = 0; i < n; i++)
    if (isB[i] && !isB[(i + 1) % n]) PA.push_back(i);
  const I32 m = (I32)PA.size();
  if (m == 0) return 0;
  // One array as the reference lays it out: buckets [0, m), merge scratch [m, n - m) (later the
  // ranks R = SA + m), the B* positions at [n - m, n).  The layout matters beyond the sizes:
  // the last doubling round reads keys R[x] with x up to 2m, i.e. scratch / position slots.
  std::vector<I32> SA(3 * (size_t)n + 16, 0);
  std::copy(PA.begin(), PA.end(), SA.begin() + (n - m));
  std::vector<I32> start(65536, 0), cnt(65536, 0);
  for (I32 j = 0; j < m; j++) cnt[(t[PA[j]] << 8) | T.at(PA[j] + 1)]++;
  {
    I32 acc = 0;
    for (int c0 = 0; c0 < 256; c0++)
      for (int c1 = c0 + 1; c1 < 256; c1++) {
        acc += cnt[(c0 << 8) | c1];
        start[(c0 << 8) | c1] = acc;  // end of the bucket, filled downwards
      }
  }
  auto bucket_of = [&](I32 j) { return (t[PA[j]] << 8) | T.at(PA[j] + 1); };
  for (I32 j = m - 2; j >= 0; --j) SA[--start[bucket_of(j)]] = j;
  SA[--start[bucket_of(m - 1)]] = m - 1;
  I32* buf = SA.data() + m;
  I32 bufsize = n - 2 * m;
  std::vector<I32> tmp(256 + 2);
  if (bufsize <= 256) {
    buf = tmp.data();
    bufsize = 256;
  }
  SubstringStage ss(T, SA.data() + (n - m), m, n);
  {
    I32 end = m;
    for (int c0 = 255; end > 0; --c0)
      for (int c1 = 255; c0 < c1; --c1) {
        const I32 b = start[(c0 << 8) | c1];
        if (end - b > 1) ss.sort_bucket(SA.data(), b, end, buf, bufsize, SA[b] == m - 1);
        end = b;
      }
  }
  // ranks: a group of equal substrings takes its last slot; runs of distinct items become
  // final runs (-length at their head)
  I32* R = SA.data() + m;
  I32* S = SA.data();
  for (I32 i = m - 1; i >= 0; --i) {
    I32 x = S[i];
    if (x >= 0) {
      const I32 j = i;
      do R[x] = i;
      while (--i >= 0 && (x = S[i]) >= 0);
      S[i + 1] = i - j;
      if (i <= 0) break;
    }
    const I32 j = i;
    do {
      S[i] = ~x;
      R[S[i]] = j;
    } while ((x = S[--i]) < 0);
    R[x] = j;
  }
  RankStage rs(S, R, m);
  rs.run(1);
  // r = rank of copy 0 of the first B* suffix among its k copies (items 0, mw, 2 mw, ...)
  const I32 k = n / p, mw = m / k;
  I32 r = 0;
  for (I32 c = 1; c < k; c++) r += R[c * mw] < R[0];
  return r;
}

// rank of rotation 0 among the p distinct rotations of the root (host, for the test entry)
I32 root_rank0(const uint8_t* t, I32 p) {
  I32 r = 0;
  for (I32 i = 1; i < p; i++) {
    I32 x = 0;
    while (x < p && t[(i + x) % p] == t[x]) x++;
    if (x < p && t[(i + x) % p] < t[x]) r++;
  }
  return r;
}

I32 primitive_period(const uint8_t* t, I32 n) {
  for (I32 p = 1; p <= n / 2; p++) {
    if (n % p) continue;
    bool ok = true;
    for (I32 i = p; i < n && ok; i++) ok = t[i] == t[i - p];
    if (ok) return p;
  }
  return n;
}

}  // namespace

// ------------------------------------------------------------------ interface
int32_t periodic_copy_rank(const uint8_t* blk, int32_t n, int32_t p) {
  if (!blk || n <= 0 || p <= 0 || n % p) throw ResolverFailure();
  if (p == n) return 0;
  return copy_rank(blk, n, p);
}

int32_t periodic_origptr(const uint8_t* blk, int32_t n) {
  if (!blk || n <= 0) throw ResolverFailure();
  const I32 p = primitive_period(blk, n);
  if (p == n) throw ResolverFailure();  // not periodic: the sort's rank is the origPtr
  if (p == 1) return 0;
  return root_rank0(blk, p) * (n / p) + copy_rank(blk, n, p);
}

void resolve_origptrs(const uint8_t* d_blk, const std::vector<uint32_t>& boff, const std::vector<uint32_t>& period,
                      std::vector<uint32_t>& rank) {
  static std::mutex mu;
  static std::map<std::string, int32_t> memo;  // identical periodic blocks resolve once per process
  const size_t nb = rank.size();
  for (size_t b = 0; b < nb; b++) {
    const uint32_t n = boff[b + 1] - boff[b], p = period[b];
    const uint32_t k = n / p;
    if (k == 1) continue;  // aperiodic: the rank is the origPtr
    if (p == 1) {          // one symbol: no B* suffix, origPtr 0 (blocksort.c:1349)
      rank[b] = 0;
      continue;
    }
    std::string bytes(n, '\0');
    if (hipMemcpy(&bytes[0], d_blk + boff[b], n, hipMemcpyDeviceToHost) != hipSuccess) throw ResolverFailure();
    int32_t r;
    {
      std::lock_guard<std::mutex> g(mu);
      auto it = memo.find(bytes);
      if (it == memo.end()) {
        if (memo.size() > 64) memo.clear();
        it = memo.emplace(bytes, copy_rank((const uint8_t*)bytes.data(), (I32)n, (I32)p)).first;
      }
      r = it->second;
    }
    rank[b] = rank[b] * k + (uint32_t)r;  // rank0 among the root's rotations, then the copy
  }
}

}  // namespace bzg
