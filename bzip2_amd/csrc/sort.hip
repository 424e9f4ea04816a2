// sort.hip -- stage A4: batched cyclic suffix sorting (BWT) for all blocks of a batch.
//
// Replaces the reference's divsufsort (blocksort.c:1503-1545).  For an aperiodic block all
// rotations are distinct, so any correct sort yields the reference's last column and
// origPtr (parity fact 3).  Periodic blocks (w^k) are reduced to their
// primitive root w; the rank of rotation 0 among the k identical copies is the copy rank of
// A5 (origptr.hip on the device, copyrank.cpp on the host).
//
// The sort is a string sort keyed directly by the block text (read through L2: a block is
// <= 900 kB and the workgroups of an XCD walk the blocks in order), not by rank arrays that
// would have to be gathered from HBM:
//   S1  MSD byte passes: every block is split into buckets by its leading characters (one
//       counting pass per character over the buckets still larger than kBig).  Buckets are
//       emitted into size-class lists (2-8, 9-16, 17-32, 33-64, 65-128, 129-256) at offsets
//       from one class-major scan per pass.
//   S2  every class is sorted by one wave per 64 / kSeg buckets: the next 8 characters of
//       each rotation are gathered, a bitonic network in registers sorts the segment by
//       (run start, key, index), unique rotations write SA / BWT byte / origPtr, and tied
//       runs repeat with the next 8 characters (2-8: rank counting on 16 characters).
//   S3  groups still equal after B.dwave characters (long repeats) or S1 buckets still larger
//       than kBig after kDBig characters go to prefix doubling (sortdbl.hip) over ISA ranks
//       built for the affected blocks only.
#include <algorithm>
#include <cstdlib>
#include <string>

#include "qsa.h"
#include "scan.h"
#include "sort_common.h"

namespace bzg {

namespace {

constexpr int kT = 256;
constexpr uint32_t kBig = 512;        // buckets larger than this are split by S1 byte passes
constexpr uint32_t kDTile = 4096;     // rotations per workgroup in a tiled S1 pass
constexpr uint32_t kPerT = kDTile / kT;
constexpr uint32_t kDBig = 16;        // S1 byte passes stop at this depth (then doubling)
constexpr uint32_t kSG = 2048;      // S1 groups up to this size are packed into shared tiles
// size classes: 0..6 go to S2 (2-8 .. 257-512), 7 / 8 to the next S1 pass (packed / tiled),
// 9 (still big after kDBig characters) to the doubling fallback
constexpr int kNCls = 9;
constexpr int kS2Cls = 7;             // classes sorted by S2
constexpr uint32_t kClsPacked = 7, kClsTiled = 8;
constexpr uint32_t kClsMax[8] = {8, 16, 32, 64, 128, 256, kBig, kSG};
constexpr uint32_t kClsDeep = 9;
// S2 workgroups walk the (block-ordered) group lists XCD by XCD: each XCD's L2 then holds the
// text and slots of its own few blocks instead of every block's
__device__ __forceinline__ uint32_t s2_wg() { return xcd_remap(blockIdx.x, gridDim.x); }

__host__ __device__ __forceinline__ uint32_t size_cls(uint32_t n) {
  return n <= 8 ? 0u : n <= 16 ? 1u : n <= 32 ? 2u : n <= 64 ? 3u : n <= 128 ? 4u : n <= 256 ? 5u : n <= kBig ? 6u
         : n <= kSG ? 7u : 8u;
}

struct SortOut {
  uint8_t* bwt;      // last column of aperiodic units, same offsets as the blocks
  uint32_t* rank0;   // slot of rotation 0 relative to its unit
  Grp* deep;         // groups left for the doubling fallback
  uint32_t* n_deep;
  Grp* tdeep;        // k_tiny<2>: the deep pair of bucket i at [i] (size 0: none; k_deep_compact_all appends them)
  Grp* dslot;        // classes 9..32: group i's deep groups at [i * dm, + dnum[i]) (k_deep_compact_all appends them)
  uint32_t* dnum;
  uint32_t dm;
  unsigned long long* dbg;  // BZG_DEBUG counters (null otherwise)
};

struct ClsLists {
  Grp* l[kNCls];
  uint32_t base[kNCls];  // entries already in each list before this pass
};

// ---------------------------------------------------------------- text access
// (v + d) mod len for v < len.
__device__ __forceinline__ uint32_t cyc_pos(uint32_t v, uint32_t d, uint32_t len) {
  uint32_t q = v + d;
  if (q >= len) {
    q -= len;
    if (q >= len) q %= len;
  }
  return q;
}

// 4 bytes at p, any alignment (one unaligned global_load_dword; every text buffer has >= 16
// bytes of padding).
__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) {
  uint32_t x;
  __builtin_memcpy(&x, p, 4);
  return x;
}
__device__ __forceinline__ uint32_t ld_be4(const uint8_t* p) { return __builtin_bswap32(ld_u32(p)); }

// The 4 characters of t[0..len) starting at q (< len) when they wrap past the unit end.
__device__ __forceinline__ uint32_t text_key4_wrap(const uint8_t* t, uint32_t len, uint32_t q) {
  uint32_t k = 0;
  for (uint32_t i = 0; i < 4; i++) k = (k << 8) | t[(q + i) % len];
  return k;
}
// Same for len >= 4 (S1 units are longer than kBig): one subtraction per character.
__device__ __forceinline__ uint32_t text_key4_wrap_long(const uint8_t* t, uint32_t len, uint32_t q) {
  uint32_t k = 0;
#pragma unroll
  for (uint32_t i = 0; i < 4; i++) {
    const uint32_t p = q + i;
    k = (k << 8) | t[p >= len ? p - len : p];
  }
  return k;
}

// The 4 characters of the cyclic unit text t[0..len) starting at q (< len).
__device__ __forceinline__ uint32_t text_key4(const uint8_t* t, uint32_t len, uint32_t q) {
  if (q + 4 <= len) return ld_be4(t + q);
  return text_key4_wrap(t, len, q);
}

// Characters q .. q + 4N - 1 of the cyclic unit text as big-endian words, one at a time
// (the wrap-around path; rare).
// (a rolled loop with an incremental index: unrolled, its 4N modulo reductions and byte loads
// set the register peak of the S2 sorts although it runs only for keys that wrap)
template <int N>
__device__ __forceinline__ void text_words_wrap(const uint8_t* t, uint32_t len, uint32_t q, uint32_t (&k)[N]) {
  uint32_t acc[N];
#pragma unroll
  for (int w = 0; w < N; w++) acc[w] = 0;
  uint32_t p = q;
#pragma unroll 1
  for (uint32_t j = 0; j < 4u * N; j++) {
    const uint32_t c = t[p];
    p = p + 1 == len ? 0u : p + 1;
#pragma unroll
    for (int w = 0; w < N; w++) acc[w] = (j >> 2) == (uint32_t)w ? (acc[w] << 8) | c : acc[w];
  }
#pragma unroll
  for (int w = 0; w < N; w++) k[w] = acc[w];
}
// The N + 1 aligned words covering characters p .. p + 4N - 1 (loads only; text_words_of
// turns them into big-endian words).  Split so that a caller issues the loads of all its
// elements before it uses any.
template <int N>
__device__ __forceinline__ void text_raw(const uint8_t* p, uint32_t (&x)[N + 1]) {
  // (pointer arithmetic, not an integer round trip, so the loads stay global_load, not flat)
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p - ((uintptr_t)p & 3u));
#pragma unroll
  for (int i = 0; i <= N; i++) x[i] = w[i];
}
template <int N>
__device__ __forceinline__ void text_words_of(const uint8_t* p, const uint32_t (&x)[N + 1], uint32_t (&k)[N]) {
  const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
#pragma unroll
  for (int i = 0; i < N; i++) k[i] = __builtin_bswap32(__builtin_amdgcn_alignbyte(x[i + 1], x[i], sh));
}

// The 16 characters starting at q, as four big-endian words.
__device__ __forceinline__ void text_key16(const uint8_t* t, uint32_t len, uint32_t q, uint32_t (&k)[4]) {
  if (q + 16 <= len) {
    const uintptr_t a = (uintptr_t)(t + q);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(t + q - (a & 3u));
    const uint32_t sh = (uint32_t)(a & 3u);  // byte shift
    const uint32_t x0 = w[0], x1 = w[1], x2 = w[2], x3 = w[3], x4 = w[4];
    k[0] = __builtin_bswap32(__builtin_amdgcn_alignbyte(x1, x0, sh));
    k[1] = __builtin_bswap32(__builtin_amdgcn_alignbyte(x2, x1, sh));
    k[2] = __builtin_bswap32(__builtin_amdgcn_alignbyte(x3, x2, sh));
    k[3] = __builtin_bswap32(__builtin_amdgcn_alignbyte(x4, x3, sh));
    return;
  }
  for (int w = 0; w < 4; w++) {
    uint32_t x = 0;
    for (uint32_t i = 0; i < 4; i++) x = (x << 8) | t[(q + 4 * w + i) % len];
    k[w] = x;
  }
}

// A rotation v of `unit` is fully ordered at global slot `slot`: SA, BWT byte, origPtr.
__device__ __forceinline__ void emit_final(const SortBufs& B, const SortOut& O, const Unit& U, uint32_t unit,
                                           uint32_t slot, uint32_t v, bool write_sa) {
  if (write_sa) B.sa[slot] = v;
  const uint32_t r = slot - U.sbase;
  if (U.k == 1) O.bwt[U.toff + r] = B.text[U.toff + (v == 0 ? U.len - 1 : v - 1)];
  if (v == 0) O.rank0[unit] = r;
}

// ---------------------------------------------------------------- setup
// Units of one rotation are done; the others are classed by size: <= kBig rotations go
// straight to S2, larger ones to the S1 byte passes.  (Few units: one atomic per wave.)
__global__ void k_init_units(const Unit* __restrict__ units, uint32_t nu, SortBufs B, SortOut O, ClsLists C,
                             uint32_t* __restrict__ ccount) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = u < nu;
  Unit U{0, 0, 0, 1};
  if (valid) U = units[u];
  if (valid && U.len == 1) emit_final(B, O, U, u, U.sbase, 0, true);
  const uint32_t c = (valid && U.len >= 2) ? size_cls(U.len) : 0xffu;
  for (int k = 0; k < kNCls; k++) {
    const uint32_t pos = wave_append(ccount + k, c == (uint32_t)k);
    if (c == (uint32_t)k) C.l[k][pos] = Grp{U.sbase, U.len, u, kGrpIdent};
  }
}

// One launch for both lists of an S1 pass: the tiled groups' tile counts (for the tile prefix
// TP) at [0, n7), then, for the packed groups, their sizes (for the element prefix P) and
// each group's unit beside it, so that a packed tile reads its groups and their units in one
// round trip instead of two dependent ones.
__global__ void k_group_prep(const Grp* __restrict__ L7, uint32_t n7, uint32_t* __restrict__ TP,
                             const Grp* __restrict__ L6, uint32_t n6, const Unit* __restrict__ units,
                             uint32_t* __restrict__ sizes, Unit* __restrict__ gunits) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n7) {
    TP[i] = ceil_div(L7[i].size, kDTile);
  } else if (i - n7 < n6) {
    const Grp gr = L6[i - n7];
    sizes[i - n7] = gr.size;
    gunits[i - n7] = units[gr.unit];
  }
}

// One record per S1 tile (TP: exclusive scan of the groups' tile counts): the tile's group,
// its unit and its position, so that a tile reads one 48-byte record instead of a chain of
// dependent loads (tile -> group -> unit; a binary search over TP before that).
struct TileRec {
  Grp g;
  Unit u;
  uint32_t gi;  // group index in the list
  uint32_t k;   // tile index within the group
  uint32_t pad[2];
};
__global__ void k_tile_owner(const Grp* __restrict__ L, uint32_t n, const uint32_t* __restrict__ TP,
                             const Unit* __restrict__ units, TileRec* __restrict__ TR) {
  const uint32_t g = blockIdx.x;  // one wave per group, lanes over its tiles
  if (g >= n) return;
  const Grp gr = L[g];
  const Unit u = units[gr.unit];
  const uint32_t t0 = TP[g], c = ceil_div(gr.size, kDTile);
  for (uint32_t k = threadIdx.x; k < c; k += blockDim.x) TR[t0 + k] = TileRec{gr, u, g, k, {0u, 0u}};
}

// LDS exchange among the lanes of one wave (LDS operations of a wave complete in order)
__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

// ---------------------------------------------------------------- S1 byte passes
// Every member of a group carries a key cache (sk / sk2 beside sa / sa2): the next characters
// of its rotation, most significant first, of which grp_cache(g) bytes are valid.  A pass
// consumes the top byte; a group whose cache is empty gathers 4 characters from the text
// (identity groups read them coalesced), so the text is read once per 4 passes.
//   k_s1_hist leaves, for an empty cache, the gathered key in
//   the source slot's cache (each member is owned by one workgroup), so that
//   k_s1_scatter finds a full cache in every non-identity slot (k_s1s_pass, which counts and
//   scatters in one kernel, refills in registers).
// Loads are issued through a selected address (cache slot or text) before any value is used,
// so a wave keeps all kPerT gathers in flight; keys that wrap past the unit end are patched
// afterwards (rare).

// Loads members [lo, hi) of group gr: rotations vv and keys kk (top byte = this pass's
// character).  Lanes past hi get a copy of member hi - 1.  kCounting: empty caches are
// refilled from the text and stored back.
template <bool kCounting>
__device__ __forceinline__ void s1_load(const SortBufs& B, const Grp& gr, const Unit& U, uint32_t lo, uint32_t hi,
                                        uint32_t (&vv)[kPerT], uint32_t (&kk)[kPerT]) {
  const bool alt = gr.flags & kGrpAlt;
  const uint32_t* src = alt ? B.sa2 : B.sa;
  uint32_t* srck = alt ? B.sk2 : B.sk;
  const bool ident = gr.flags & kGrpIdent;
  const uint32_t depth = grp_depth(gr);
  const bool fresh = ident || (kCounting && grp_cache(gr) == 0);
  const uint8_t* ut = B.text + U.toff;
  // (whole-loop uniform branches keep vv / kk in registers)
  if (ident) {
#pragma unroll
    for (int i = 0; i < (int)kPerT; i++) vv[i] = min(lo + i * kT + threadIdx.x, hi - 1);
  } else if (!kCounting || fresh) {  // the histogram of a full cache needs no rotations
#pragma unroll
    for (int i = 0; i < (int)kPerT; i++) vv[i] = src[gr.start + min(lo + i * kT + threadIdx.x, hi - 1)];
  }
  if (!fresh) {
#pragma unroll
    for (int i = 0; i < (int)kPerT; i++) kk[i] = srck[gr.start + min(lo + i * kT + threadIdx.x, hi - 1)];
  }
  if (fresh) {
#pragma unroll
    for (int i = 0; i < (int)kPerT; i++) kk[i] = ld_u32(ut + cyc_pos(vv[i], depth, U.len));
#pragma unroll
    for (int i = 0; i < (int)kPerT; i++) {
      const uint32_t q = cyc_pos(vv[i], depth, U.len);
      kk[i] = q + 4 <= U.len ? __builtin_bswap32(kk[i]) : text_key4_wrap_long(ut, U.len, q);
    }
    if (kCounting && !ident) {
#pragma unroll
      for (int i = 0; i < (int)kPerT; i++) {
        const uint32_t e = lo + i * kT + threadIdx.x;
        if (e < hi) srck[gr.start + e] = kk[i];
      }
    }
  }
}

// cache bytes valid in the buckets of a group after this pass
__device__ __forceinline__ uint32_t s1_next_cache(const Grp& gr) {
  const uint32_t c = (gr.flags & kGrpIdent) ? 0u : grp_cache(gr);
  return c ? c - 1 : 3u;
}
// the same for the buckets of a tiled pass
__device__ __forceinline__ uint32_t tiled_next_cache(const Grp& gr) { return s1_next_cache(gr); }

constexpr uint32_t kHistCp = 4;  // (8 copies measured neutral: profiles/r04_ab_*)

__global__ void __launch_bounds__(kT) k_s1_hist(const TileRec* __restrict__ TR, SortBufs B, uint32_t* __restrict__ hist) {
  // kHistCp copies of every bin in consecutive words (lane % kHistCp picks one): lanes of a
  // wave that count the same character (skewed text) hit several banks instead of one word
  __shared__ uint32_t h[256 * kHistCp];
  const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
  const TileRec tr = TR[t];
  const Grp gr = tr.g;
  const Unit U = tr.u;
  const uint32_t lo = tr.k * kDTile, hi = min(gr.size, lo + kDTile);
#pragma unroll
  for (int q = 0; q < (int)kHistCp; q++) h[q * kT + threadIdx.x] = 0;
  uint32_t vv[kPerT], kk[kPerT];
  s1_load<true>(B, gr, U, lo, hi, vv, kk);
  __syncthreads();
  const uint32_t cp = threadIdx.x % kHistCp;
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++)
    if (lo + i * kT + threadIdx.x < hi) atomicAdd(&h[(kk[i] >> 24) * kHistCp + cp], 1u);
  __syncthreads();
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < (int)kHistCp; q += 4) {
    const uint4 c4 = reinterpret_cast<const uint4*>(h)[threadIdx.x * (kHistCp / 4) + q / 4];
    c += c4.x + c4.y + c4.z + c4.w;
  }
  hist[(size_t)t * 256 + threadIdx.x] = c;
}

__device__ __forceinline__ uint32_t bucket_cls(uint32_t total, uint32_t depth) {
  if (total < 2) return 0xffu;
  const uint32_t c = size_cls(total);
  return (c >= kClsPacked && depth >= kDBig) ? kClsDeep : c;
}

// One workgroup per group: bucket totals and bases, per-tile offsets, and the number of
// buckets of every size class (class-major: ccnt[c * nG + g]).
__global__ void __launch_bounds__(kT) k_s1_off(const Grp* __restrict__ G, uint32_t nTot, const uint32_t* __restrict__ TP,
                                               uint32_t* __restrict__ hist, uint32_t* __restrict__ tot,
                                               uint32_t* __restrict__ ccnt, Grp* __restrict__ deep,
                                               uint32_t* __restrict__ n_deep) {
  __shared__ uint32_t sh[kT / 64];
  __shared__ uint32_t cc[kNCls + 1];
  const uint32_t g = blockIdx.x;
  const Grp gr = G[g];
  const uint32_t t0 = TP[g], t1 = t0 + ceil_div(gr.size, kDTile);
  const uint32_t d = threadIdx.x;
  if (d <= (uint32_t)kNCls) cc[d] = 0;
  // kOffBatch tiles' counts are loaded before any is used (a group of the first pass has ~440
  // tiles: one dependent load per tile was ~0.4 ms per pass)
  constexpr uint32_t kOffBatch = 16;
  uint32_t total = 0;
  for (uint32_t t = t0; t < t1; t += kOffBatch) {
    uint32_t c[kOffBatch];
#pragma unroll
    for (uint32_t k = 0; k < kOffBatch; k++) c[k] = t + k < t1 ? hist[(size_t)(t + k) * 256 + d] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < kOffBatch; k++) total += c[k];
  }
  const uint32_t incl = block_incl_sum(total, sh, (uint32_t*)nullptr);
  const uint32_t base = gr.start + incl - total;
  tot[(size_t)g * 256 + d] = total;
  uint32_t run = base;
  for (uint32_t t = t0; t < t1; t += kOffBatch) {
    uint32_t c[kOffBatch];
#pragma unroll
    for (uint32_t k = 0; k < kOffBatch; k++) c[k] = t + k < t1 ? hist[(size_t)(t + k) * 256 + d] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < kOffBatch; k++) {
      if (t + k < t1) hist[(size_t)(t + k) * 256 + d] = run;
      run += c[k];
    }
  }
  const uint32_t depth = grp_depth(gr) + 1;
  const uint32_t cl = bucket_cls(total, depth);
#pragma unroll
  for (int k = 0; k < kNCls; k++) {
    const uint32_t n = (uint32_t)__popcll(__ballot(cl == (uint32_t)k));
    if (__lane_id() == 0 && n) atomicAdd(&cc[k], n);
  }
  if (cl == kClsDeep) {  // rare: a bucket still larger than kBig after kDBig characters
    const uint32_t dst_alt = (gr.flags & kGrpIdent) ? 0u : ((gr.flags & kGrpAlt) ^ 1u);
    deep[wave_append(n_deep, true)] = Grp{base, total, gr.unit, grp_flags(dst_alt, depth, tiled_next_cache(gr))};
  }
  __syncthreads();
  if (d < (uint32_t)kNCls) ccnt[(size_t)d * nTot + g] = cc[d];
}

// Scatter of one tile into the bucket order; the first tile of a group also emits the
// group's buckets into the class lists (cscan: exclusive scan of ccnt).  The tile is first
// reordered by bucket in LDS, so the global stores run along each bucket's range.
__global__ void __launch_bounds__(kT) k_s1_scatter(const TileRec* __restrict__ TR,
                                                   SortBufs B, SortOut O, const uint32_t* __restrict__ off,
                                                   const uint32_t* __restrict__ tot, const uint32_t* __restrict__ cscan,
                                                   uint32_t nTot, ClsLists C) {
  // 36 KB of LDS (4 workgroups per CU): the bucket counters (4 bank-spread copies per bucket,
  // see k_s1_hist) and the reordered tile, rotations and key caches.  Once the tile is
  // reordered the counter space holds each bucket's store base and flags (and the emission's
  // wave counts); the scan scratch lives in the tile space before the tile is.  (Round 3 fitted
  // 2048-rotation tiles in 20 KB for 8 workgroups; 4096-rotation tiles measured faster in round
  // 4, and one shared 16 KB reorder array, or 7 waves per SIMD, gave nothing in round 6:
  // profiles/r06_ab_s1_scatter.txt.)
  __shared__ uint32_t cnt[256 * 4];
  __shared__ uint32_t Lv[kDTile], Lk[kDTile];
  static_assert(kDTile == kPerT * kT, "one element per thread and round");
  uint32_t* const base = cnt;          // after the reorder: global slot of the bucket's first element - its LDS start
  uint32_t* const flag = cnt + 256;    // bit 0: a bucket of one; bit 1: the bucket stays in S1 (needs its key caches)
  uint32_t* const wcnt = cnt + 512;    // [wave][class] counts of the bucket emission
  const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
  const TileRec tr = TR[t];
  const uint32_t g = tr.gi;
  const Grp gr = tr.g;
  const Unit U = tr.u;
  const uint32_t lo = tr.k * kDTile, hi = min(gr.size, lo + kDTile);
  const bool dst_alt = !(gr.flags & kGrpIdent) && !(gr.flags & kGrpAlt);
  uint32_t* dst = dst_alt ? B.sa2 : B.sa;
  uint32_t* dstk = dst_alt ? B.sk2 : B.sk;
  const uint32_t d = threadIdx.x;
  const uint32_t total = tot[(size_t)g * 256 + d];
  const uint32_t gbase = off[(size_t)t * 256 + d];
#pragma unroll
  for (int q = 0; q < 4; q++) cnt[q * kT + d] = 0;
  // (a cache that this pass empties is not stored: the next pass refills it from the text)
  const uint32_t myflag = (total == 1 ? 1u : 0u) |
                          (bucket_cls(total, grp_depth(gr) + 1) >= kClsPacked &&
                           bucket_cls(total, grp_depth(gr) + 1) <= kClsTiled && tiled_next_cache(gr) ? 2u : 0u);
  uint32_t vv[kPerT], kk[kPerT];
  s1_load<false>(B, gr, U, lo, hi, vv, kk);
  __syncthreads();
  uint32_t rk[kPerT];
  const uint32_t cp = threadIdx.x & 3u;
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++)
    if (lo + i * kT + threadIdx.x < hi) rk[i] = atomicAdd(&cnt[(kk[i] >> 24) * 4 + cp], 1u);
  __syncthreads();
  uint32_t mybase;
  {  // bucket d's LDS start, and the start of each of its copies (any order within a bucket)
    const uint4 c4 = reinterpret_cast<const uint4*>(cnt)[d];
    const uint32_t c = c4.x + c4.y + c4.z + c4.w;
    const uint32_t lstart = block_incl_sum(c, Lv, (uint32_t*)nullptr) - c;
    reinterpret_cast<uint4*>(cnt)[d] =
        make_uint4(lstart, lstart + c4.x, lstart + c4.x + c4.y, lstart + c4.x + c4.y + c4.z);
    mybase = gbase - lstart;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++) {
    if (lo + i * kT + threadIdx.x < hi) {
      const uint32_t lp = cnt[(kk[i] >> 24) * 4 + cp] + rk[i];
      Lv[lp] = vv[i];
      Lk[lp] = kk[i];
    }
  }
  __syncthreads();
  base[d] = mybase;
  flag[d] = myflag;
  __syncthreads();
  const uint32_t m = hi - lo;
  uint32_t pos[kPerT];
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++) {
    const uint32_t x = i * kT + threadIdx.x;
    if (x < m) {
      vv[i] = Lv[x];
      kk[i] = Lk[x];
      pos[i] = base[kk[i] >> 24] + x;
      dst[pos[i]] = vv[i];
      if (flag[kk[i] >> 24] & 2u) dstk[pos[i]] = kk[i] << 8;
    }
  }
  // a bucket of one: this rotation is ordered (its primary-SA copy is made by s1_single,
  // since other workgroups may still read the primary SA in this pass)
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++)
    if (i * kT + threadIdx.x < m && (flag[kk[i] >> 24] & 1u)) emit_final(B, O, U, gr.unit, pos[i], vv[i], !dst_alt);
  if (tr.k != 0) return;
  // ---- bucket emission (digit order within the group)
  const uint32_t depth = grp_depth(gr) + 1;
  const uint32_t cl = bucket_cls(total, depth);
  const uint32_t w = d >> 6;
  uint32_t rank = 0;
#pragma unroll
  for (int k = 0; k < kNCls; k++) {
    const uint64_t mk = __ballot(cl == (uint32_t)k);
    if (cl == (uint32_t)k) rank = (uint32_t)__popcll(mk & lanemask_lt());
    if (__lane_id() == 0) wcnt[w * kNCls + k] = (uint32_t)__popcll(mk);
  }
  __syncthreads();
  if (cl < (uint32_t)kNCls) {
    for (uint32_t x = 0; x < w; x++) rank += wcnt[x * kNCls + cl];
    const uint32_t p = C.base[cl] + cscan[(size_t)cl * nTot + g] - cscan[(size_t)cl * nTot] + rank;
    C.l[cl][p] = Grp{gbase, total, gr.unit, grp_flags(dst_alt ? kGrpAlt : 0u, depth, tiled_next_cache(gr))};
  }
}

// The primary-SA copies of the buckets of one that a tiled pass left in the alternate SA
// (one workgroup per tiled group; the launch is shared with s1s_emit, see k_s1_tail).
__device__ __forceinline__ void s1_single(const Grp* __restrict__ G, SortBufs B, const uint32_t* __restrict__ tot,
                                          uint32_t g) {
  __shared__ uint32_t sh[kT / 64];
  const Grp gr = G[g];
  if ((gr.flags & kGrpIdent) || (gr.flags & kGrpAlt)) return;  // pass wrote the primary SA
  const uint32_t total = tot[(size_t)g * 256 + threadIdx.x];
  const uint32_t incl = block_incl_sum(total, sh, (uint32_t*)nullptr);
  const uint32_t s = gr.start + incl - total;
  if (total == 1) B.sa[s] = B.sa2[s];
}


// ---- packed S1 tiles: groups of kBig+1 .. kSG rotations, several per workgroup (all the
// groups whose element prefix falls in a kSG window; <= kSGrp groups, < 2 kSG rotations).
// A group lies in one tile, so its counts, bases and scatter stay in LDS, and singletons can
// write the primary SA directly.  Two kernels per pass: counts of buckets per size class
// (for the class-major scan), then the scatter and bucket emission; both take the pass's
// character from the key caches (the first refills empty caches of non-identity groups).
constexpr uint32_t kSGrp = kSG / (kBig + 1) + 2;

// tile index of item i = P[i] / kSG; mark the first item of each tile and one past its last.
// Groups hold at most kSG rotations, so every window of kSG prefix positions holds a group
// start but the last window(s) after the last start: those tiles (up to ceil(total / kSG),
// total = *ptotal) are marked empty here.
__global__ void k_tile_first(const uint32_t* __restrict__ P, uint32_t n, const uint32_t* __restrict__ ptotal,
                             uint32_t* __restrict__ first, uint32_t* __restrict__ last) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t t = P[i] / kSG;
  if (i == 0 || P[i - 1] / kSG != t) first[t] = i;
  if (i == n - 1 || P[i + 1] / kSG != t) last[t] = i + 1;
  if (i == n - 1)
    for (uint32_t e = t + 1; e < ceil_div(*ptotal, kSG); e++) first[e] = 0xffffffffu;
}


// packed kernels: 512 threads x 8 elements (a tile holds < 2 kSG rotations; kSG on average,
// so the element loops stop at the tile's last 512-element round)
constexpr uint32_t kTS = 512, kPerTS = 2 * kSG / kTS;
// (group, digit) bins keep kCp copies in consecutive words (thread & 1 picks one), as in k_s1_hist
constexpr uint32_t kCp = 2;
struct S1sLds {
  // (group, digit) bins: counts, then (in place) exclusive tile-relative bases; entry
  // ni * 256 = tile size, so a bin's total is the difference of neighbouring entries
  uint32_t cur[kSGrp * 256 * kCp + 1];
  // per group: first slot, tile offset, flags, unit, and the unit's text offset, length,
  // first slot and copies
  uint32_t gstart[kSGrp], goff[kSGrp + 1], gfl[kSGrp], gunit[kSGrp], gtoff[kSGrp], glen[kSGrp], gsb[kSGrp], gk[kSGrp];
  uint32_t sh[kTS / 64];
  uint32_t cc[kNCls + 1];
};

// Loads the tile's groups; returns the number of groups (0: empty tile).
__device__ __forceinline__ uint32_t s1s_setup(S1sLds& S, const Grp* __restrict__ SG, const Unit* __restrict__ GU,
                                              const uint32_t* __restrict__ first, const uint32_t* __restrict__ last,
                                              uint32_t t) {
  const uint32_t i0 = first[t];
  if (i0 == 0xffffffffu) return 0;
  const uint32_t ni = min(last[t], i0 + kSGrp) - i0;
  if (threadIdx.x < ni) {
    const Grp g = SG[i0 + threadIdx.x];
    const Unit U = GU[i0 + threadIdx.x];
    S.gstart[threadIdx.x] = g.start;
    S.goff[threadIdx.x + 1] = g.size;
    S.gfl[threadIdx.x] = g.flags;
    S.gunit[threadIdx.x] = g.unit;
    S.gtoff[threadIdx.x] = U.toff;
    S.glen[threadIdx.x] = U.len;
    S.gsb[threadIdx.x] = U.sbase;
    S.gk[threadIdx.x] = U.k;
  }
  for (uint32_t i = threadIdx.x; i < ni * 256 * kCp; i += kTS) S.cur[i] = 0;
  if (threadIdx.x <= (uint32_t)kNCls) S.cc[threadIdx.x] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    S.goff[0] = 0;
    for (uint32_t j = 1; j <= ni; j++) S.goff[j] += S.goff[j - 1];
  }
  __syncthreads();
  return ni;
}

// Group boundaries of the tile in scalar registers (goff[q], or ~0 past the last group): the
// owner of a tile element is a compare per group boundary of the tile (scalar loop bound).
struct S1sOwner {
  uint32_t go[kSGrp - 1];
  uint32_t nb;  // boundaries in use (ni - 1)
  __device__ __forceinline__ S1sOwner(const S1sLds& S, uint32_t ni) : nb(ni - 1) {
#pragma unroll
    for (uint32_t q = 1; q < kSGrp; q++) go[q - 1] = __builtin_amdgcn_readfirstlane(q < ni ? S.goff[q] : 0xffffffffu);
  }
  __device__ __forceinline__ uint32_t operator()(uint32_t e) const {
    uint32_t j = 0;
#pragma unroll
    for (uint32_t q = 0; q + 1 < kSGrp; q++) {
      if (q >= nb) break;  // uniform
      j += e >= go[q];
    }
    return j;
  }
};

// One packed pass in one kernel: counts, LDS reorder, stores of the slots and caches, and
// the tile's buckets of two or more rotations as records (group:5 | start:13 | size:14,
// tile-relative) in the tile's own part of `rec` (it starts at half the tile's first element
// offset: a tile of n rotations has at most n / 2 such buckets), with the per-class counts for
// the class-major scan.  s1s_emit (k_s1_tail) turns the records into class-list entries.
// Element rounds past the tile's size are skipped (uniform branches); loads are issued for
// all rounds before their values are used, from addresses selected without branches.
__device__ __forceinline__ uint32_t rec_pack(uint32_t j, uint32_t start, uint32_t size) {
  return (j << 27) | (start << 14) | size;  // group:5 | start:13 | size:14 (tiles < 8192 rotations)
}
static_assert(kSGrp <= 32 && 2 * kSG <= 8192, "packed bucket records");
__global__ void __launch_bounds__(kTS) BZG_SGPR_LIMIT k_s1s_pass(const Grp* __restrict__ SG, const Unit* __restrict__ GU,
                                                 const uint32_t* __restrict__ first,
                                                 const uint32_t* __restrict__ last, const uint32_t* __restrict__ P,
                                                 SortBufs B, SortOut O, uint32_t* __restrict__ rec,
                                                 uint32_t* __restrict__ nrec, uint32_t* __restrict__ ccnt, uint32_t nTot,
                                                 uint32_t ibase) {
  __shared__ S1sLds S;
  __shared__ uint32_t Lv[2 * kSG];  // the tile's rotations in bucket order
  __shared__ uint32_t nr;
  const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t ni = s1s_setup(S, SG, GU, first, last, t);
  if (ni == 0) {
    if (threadIdx.x < (uint32_t)kNCls) ccnt[(size_t)threadIdx.x * nTot + ibase + t] = 0;
    if (threadIdx.x == 0) nrec[t] = 0;
    return;
  }
  if (threadIdx.x == 0) nr = 0;
  const uint32_t n = S.goff[ni];
  const uint32_t rounds = ceil_div(n, kTS);  // uniform
  const S1sOwner own(S, ni);
  const uint32_t lane = __lane_id();
  const uint32_t cp = threadIdx.x & (kCp - 1);
  uint32_t vv[kPerTS], kk[kPerTS], jj[kPerTS], qq[kPerTS];
  // rotations (identity groups: the offset; slots of identity groups hold stale values,
  // loaded anyway so that no load sits behind a branch)
#pragma unroll
  for (int i = 0; i < (int)kPerTS; i++) {
    if ((uint32_t)i >= rounds) break;
    const uint32_t e = min(i * kTS + threadIdx.x, n - 1);
    const uint32_t j = own(e), fl = S.gfl[j];
    jj[i] = j;
    qq[i] = e - S.goff[j];
    vv[i] = ((fl & kGrpAlt) ? B.sa2 : B.sa)[S.gstart[j] + qq[i]];
  }
  // keys: the cache, or 4 characters of the text when the cache is empty (loading the cache
  // words beside the slot loads instead measured no faster: profiles/r05_ab_*)
#pragma unroll
  for (int i = 0; i < (int)kPerTS; i++) {
    if ((uint32_t)i >= rounds) break;
    const uint32_t j = jj[i], fl = S.gfl[j], o = qq[i];
    if (fl & kGrpIdent) vv[i] = o;
    const bool fresh = (fl & kGrpIdent) || grp_cache(Grp{0, 0, 0, fl}) == 0;
    const uint32_t q = cyc_pos(vv[i], fl >> kGrpDepthShift, S.glen[j]);
    qq[i] = fresh ? q : 0xffffffffu;  // text position, or none
    kk[i] = ld_u32(fresh ? B.text + S.gtoff[j] + q
                         : reinterpret_cast<const uint8_t*>(((fl & kGrpAlt) ? B.sk2 : B.sk) + S.gstart[j] + o));
  }
#pragma unroll
  for (int i = 0; i < (int)kPerTS; i++) {
    if ((uint32_t)i >= rounds) break;
    if (qq[i] != 0xffffffffu) {
      const uint32_t j = jj[i];
      kk[i] = qq[i] + 4 <= S.glen[j] ? __builtin_bswap32(kk[i]) : text_key4_wrap_long(B.text + S.gtoff[j], S.glen[j], qq[i]);
    }
  }
  // counts; qq = rank of the element in its bin
#pragma unroll
  for (int i = 0; i < (int)kPerTS; i++) {
    if ((uint32_t)i >= rounds) break;
    if (i * kTS + threadIdx.x < n) qq[i] = atomicAdd(&S.cur[(jj[i] * 256 + (kk[i] >> 24)) * kCp + cp], 1u);
  }
  __syncthreads();
  // tile-relative bin bases: exclusive scan over the (group, digit) bins, in place
  {
    constexpr uint32_t kB = (kSGrp * 256 * kCp + kTS - 1) / kTS;
    uint32_t c[kB], sum = 0;
#pragma unroll
    for (int q = 0; q < (int)kB; q++) {
      const uint32_t b = threadIdx.x * kB + q;
      c[q] = b < ni * 256 * kCp ? S.cur[b] : 0u;
      sum += c[q];
    }
    uint32_t run = block_incl_sum(sum, S.sh, (uint32_t*)nullptr) - sum;
#pragma unroll
    for (int q = 0; q < (int)kB; q++) {
      const uint32_t b = threadIdx.x * kB + q;
      if (b < ni * 256 * kCp) S.cur[b] = run;
      run += c[q];
    }
    if (threadIdx.x == 0) S.cur[ni * 256 * kCp] = n;
  }
  __syncthreads();
  // bucket records (one LDS atomic per wave) and class counts
  uint32_t* trec = rec + P[first[t]] / 2;
  for (uint32_t b0 = 0; b0 < ni * 256; b0 += kTS) {
    const uint32_t b = b0 + threadIdx.x;
    const uint32_t j = b >> 8, total = b < ni * 256 ? S.cur[(b + 1) * kCp] - S.cur[b * kCp] : 0u;
    const uint32_t cl = total < 2 ? 0xffu : bucket_cls(total, grp_depth(Grp{0, 0, 0, S.gfl[j]}) + 1);
    const uint64_t m = __ballot(cl != 0xffu);
    if (m == 0) continue;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&nr, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, 0, 64);
    if (cl != 0xffu) {
      trec[base + (uint32_t)__popcll(m & lanemask_lt())] = rec_pack(j, S.cur[b * kCp], total);
      if (cl < (uint32_t)kNCls) atomicAdd(&S.cc[cl], 1u);
    }
  }
  // every element at its place: the rotation into the LDS tile (stored coalesced below), the
  // key cache of a bucket that stays in S1, and a bucket of one is final (the group lies in
  // this tile, so its primary SA slots are free)
#pragma unroll
  for (int i = 0; i < (int)kPerTS; i++) {
    if ((uint32_t)i >= rounds) break;
    if (i * kTS + threadIdx.x < n) {
      const uint32_t j = jj[i], fl = S.gfl[j];
      const uint32_t bin = j * 256 + (kk[i] >> 24);
      const uint32_t x = S.cur[bin * kCp + cp] + qq[i], total = S.cur[(bin + 1) * kCp] - S.cur[bin * kCp];
      const uint32_t v = vv[i];
      Lv[x] = v;
      const uint32_t slot = S.gstart[j] + x - S.goff[j];
      const bool dst_alt = !(fl & kGrpIdent) && !(fl & kGrpAlt);
      // key caches only for buckets that stay in S1 (S2 and S3 read the text), and only when
      // this pass leaves a byte in them
      if (bucket_cls(total, grp_depth(Grp{0, 0, 0, fl}) + 1) == kClsPacked && s1_next_cache(Grp{0, 0, 0, fl}))
        (dst_alt ? B.sk2 : B.sk)[slot] = kk[i] << 8;
      if (total == 1) {
        if (dst_alt) B.sa[slot] = v;
        const uint32_t r = slot - S.gsb[j];
        const uint32_t len = S.glen[j];
        if (S.gk[j] == 1) O.bwt[S.gtoff[j] + r] = B.text[S.gtoff[j] + (v == 0 ? len - 1 : v - 1)];
        if (v == 0) O.rank0[S.gunit[j]] = r;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < (uint32_t)kNCls) ccnt[(size_t)threadIdx.x * nTot + ibase + t] = S.cc[threadIdx.x];
  if (threadIdx.x == 0) nrec[t] = nr;
#pragma unroll
  for (int i = 0; i < (int)kPerTS; i++) {
    if ((uint32_t)i >= rounds) break;
    const uint32_t x = i * kTS + threadIdx.x;
    if (x < n) {
      const uint32_t j = own(x), fl = S.gfl[j];
      const bool dst_alt = !(fl & kGrpIdent) && !(fl & kGrpAlt);
      (dst_alt ? B.sa2 : B.sa)[S.gstart[j] + x - S.goff[j]] = Lv[x];
    }
  }
}

// The records of k_s1s_pass into the class lists (class-major offsets from cscan) or the
// deep list; one wave per tile (workgroup wg of the emission).
struct S1sEmitArgs {
  const Grp* SG;
  const uint32_t *first, *last, *P;
  uint32_t nT;
  const uint32_t *rec, *nrec;
  uint32_t ibase;
};
__device__ __forceinline__ void s1s_emit(const S1sEmitArgs& A, SortOut O, const uint32_t* __restrict__ cscan,
                                         uint32_t nTot, const ClsLists& C, uint32_t wg) {
  const Grp* __restrict__ SG = A.SG;
  const uint32_t* __restrict__ first = A.first;
  const uint32_t* __restrict__ last = A.last;
  const uint32_t* __restrict__ P = A.P;
  const uint32_t* __restrict__ rec = A.rec;
  const uint32_t* __restrict__ nrec = A.nrec;
  const uint32_t nT = A.nT, ibase = A.ibase;
  __shared__ uint32_t Wg[kT / 64][4][kSGrp];
  __shared__ uint32_t Wcc[kT / 64][kNCls];
  const uint32_t wv = threadIdx.x >> 6, lane = __lane_id();
  uint32_t* gstart = Wg[wv][0];
  uint32_t* goff = Wg[wv][1];
  uint32_t* gfl = Wg[wv][2];
  uint32_t* gunit = Wg[wv][3];
  uint32_t* cc = Wcc[wv];
  const uint32_t t = wg * (kT / 64) + wv;
  if (t >= nT) return;
  const uint32_t i0 = first[t];
  if (i0 == 0xffffffffu) return;
  const uint32_t ni = min(last[t], i0 + kSGrp) - i0;
  if (lane < ni) {
    const Grp g = SG[i0 + lane];
    gstart[lane] = g.start;
    goff[lane] = P[i0 + lane] - P[i0];
    gfl[lane] = g.flags;
    gunit[lane] = g.unit;
  }
  if (lane < (uint32_t)kNCls) cc[lane] = 0;
  wave_sync();
  const uint32_t* trec = rec + P[i0] / 2;
  const uint32_t m = nrec[t];
  for (uint32_t x = lane; x < m; x += 64) {
    const uint32_t r = trec[x];
    const uint32_t j = r >> 27, start = (r >> 14) & 0x1fffu, total = r & 0x3fffu;
    const uint32_t fl = gfl[j];
    const uint32_t depth = grp_depth(Grp{0, 0, 0, fl}) + 1;
    const uint32_t cl = bucket_cls(total, depth);
    const uint32_t dst_alt = (fl & kGrpIdent) ? 0u : ((fl & kGrpAlt) ^ 1u);
    const Grp nb{gstart[j] + start - goff[j], total, gunit[j], grp_flags(dst_alt, depth, s1_next_cache(Grp{0, 0, 0, fl}))};
    if (cl == kClsDeep) {
      O.deep[wave_append(O.n_deep, true)] = nb;
    } else {
      const uint32_t q = atomicAdd(&cc[cl], 1u);
      C.l[cl][C.base[cl] + cscan[(size_t)cl * nTot + ibase + t] - cscan[(size_t)cl * nTot] + q] = nb;
    }
  }
}

// The end of an S1 pass in one launch: workgroups [0, n7) make the tiled groups' primary-SA
// copies (s1_single), the rest turn the packed tiles' records into list entries (s1s_emit).
__global__ void __launch_bounds__(kT) k_s1_tail(const Grp* __restrict__ G7, uint32_t n7, SortBufs B,
                                               const uint32_t* __restrict__ tot, S1sEmitArgs A, SortOut O,
                                               const uint32_t* __restrict__ cscan, uint32_t nTot, ClsLists C) {
  if (blockIdx.x < n7) s1_single(G7, B, tot, blockIdx.x);
  else s1s_emit(A, O, cscan, nTot, C, blockIdx.x - n7);
}


// ---------------------------------------------------------------- S2

// The 8 characters starting at q (< len) as two big-endian words.
__device__ __forceinline__ void text_key8(const uint8_t* t, uint32_t len, uint32_t q, uint32_t& hi, uint32_t& lo) {
  if (q + 8 <= len) {
    const uintptr_t a = (uintptr_t)(t + q);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(t + q - (a & 3u));
    const uint32_t sh = (uint32_t)(a & 3u);
    const uint32_t x0 = w[0], x1 = w[1], x2 = w[2];
    hi = __builtin_bswap32(__builtin_amdgcn_alignbyte(x1, x0, sh));
    lo = __builtin_bswap32(__builtin_amdgcn_alignbyte(x2, x1, sh));
    return;
  }
  uint32_t x = 0, y = 0;
  for (uint32_t i = 0; i < 4; i++) x = (x << 8) | t[(q + i) % len];
  for (uint32_t i = 4; i < 8; i++) y = (y << 8) | t[(q + i) % len];
  hi = x;
  lo = y;
}

// The value of lane ^ M (M = 1..7) of this lane's aligned 8-lane group, by DPP only (no LDS
// traffic): quad permutes of v, or of its half-row mirror hm = g8_mirror(v) (lane ^ 7).
__device__ __forceinline__ uint32_t g8_mirror(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
}
template <int M>
__device__ __forceinline__ uint32_t g8_xor(uint32_t v, uint32_t hm) {
  static_assert(M >= 1 && M <= 7, "partner within the 8-lane group");
  constexpr int kQuad = (M & 3) == 1 ? 0xB1 : (M & 3) == 2 ? 0x4E : 0x1B;  // quad xor 1 / 2 / 3
  if constexpr (M == 7) return hm;
  else if constexpr (M < 4) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kQuad, 0xF, 0xF, false);
  else {  // lane ^ M = (lane ^ 7) ^ (M ^ 7)
    constexpr int kQ = (M ^ 7) == 1 ? 0xB1 : (M ^ 7) == 2 ? 0x4E : 0x1B;
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)hm, kQ, 0xF, 0xF, false);
  }
}

// Buckets of two rotations (most tiny buckets; long repeats make tens of millions of them)
// go to a kernel with 2 lanes per bucket, the others to 8 lanes per bucket.
// One workgroup per kSplitPer * kT list entries (thread t: entries [t * kSplitPer, ...) of the
// workgroup's range, so both outputs keep the list order) and one atomic per output per
// workgroup: single-address device atomics cost ~10 ns each, one per wave was 5 ms per GB.
constexpr uint32_t kSplitPer = 16;
__global__ void __launch_bounds__(kT) BZG_SGPR_LIMIT k_split_pairs(const Grp* __restrict__ L, uint32_t n, Grp* __restrict__ pairs,
                                                    Grp* __restrict__ rest, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t sh[kT / 64];
  __shared__ uint32_t base[2];
  const uint32_t i0 = (blockIdx.x * kT + threadIdx.x) * kSplitPer;
  Grp g[kSplitPer];
  uint32_t np = 0, nr = 0;
#pragma unroll
  for (uint32_t k = 0; k < kSplitPer; k++) {
    g[k] = i0 + k < n ? L[i0 + k] : Grp{0, 0, 0, 0};
    np += (i0 + k < n && g[k].size == 2) ? 1u : 0u;
    nr += (i0 + k < n && g[k].size != 2) ? 1u : 0u;
  }
  uint32_t tp, tr;
  const uint32_t ep = block_incl_sum(np, sh, &tp) - np;
  const uint32_t er = block_incl_sum(nr, sh, &tr) - nr;
  if (threadIdx.x == 0) {
    base[0] = tp ? atomicAdd(cnt, tp) : 0u;
    base[1] = tr ? atomicAdd(cnt + 1, tr) : 0u;
  }
  __syncthreads();
  uint32_t p = base[0] + ep, r = base[1] + er;
#pragma unroll
  for (uint32_t k = 0; k < kSplitPer; k++) {
    if (i0 + k < n) {
      if (g[k].size == 2) pairs[p++] = g[k];
      else rest[r++] = g[k];
    }
  }
}

// ---- tiny buckets: lane l takes rotation l % kW of bucket (64 / kW) * wave + l / kW.  Every step
// compares the next 16 characters with the rotations of its bucket still tied with it
// (same class, named by its first lane) and adds the smaller ones to its position.
template <int kW>
__global__ void __launch_bounds__(kT) k_tiny(const Grp* __restrict__ tiny, uint32_t n_tiny, SortBufs B, SortOut O) {
  static_assert(kW == 2 || kW == 8, "lanes per bucket");
  const uint32_t lane = __lane_id();
  const uint32_t wv = s2_wg() * (kT / 64) + (threadIdx.x >> 6);
  const uint32_t bi = wv * (64 / kW) + lane / kW, el = lane % kW;
  bool act = false;
  uint32_t s0 = 0, d = 0, v = 0, unit = 0;
  if (bi < n_tiny) {
    const Grp g = tiny[bi];
    if (el < g.size) {
      act = true;
      s0 = g.start;
      d = grp_depth(g);
      unit = g.unit;
      v = (g.flags & kGrpIdent) ? el : ((g.flags & kGrpAlt) ? B.sa2 : B.sa)[s0 + el];
    }
  }
  if (!__ballot(act)) return;
  if constexpr (kW == 8) {
    if (bi < n_tiny && el == 0) O.dnum[bi] = 0;  // (the deep branch counts the bucket's deep groups)
  } else {
    if (bi < n_tiny && el == 0) O.tdeep[bi] = Grp{0, 0, 0, 0};  // (the deep branch writes the pair's group)
  }
  Unit U{0, 1, 0, 1};
  if (act) U = B.units[unit];
  const uint8_t* t = B.text + U.toff;
  uint8_t lastc = 0;  // BWT byte of this rotation, loaded with the first key
  if (act) lastc = t[v == 0 ? U.len - 1 : v - 1];
  bool done = !act;
  uint32_t cls = act ? (lane & ~(uint32_t)(kW - 1)) : 0xffffffffu;
  uint32_t pos = 0;
  bool pos_step = false;  // a 16-character step has been taken (pairs still live are tied)
  for (;;) {
    const uint64_t live = __ballot(!done);
    if (live == 0) break;
    // still tied after B.dwave characters: leave to the doubling fallback.  The members of a
    // class and their ranks come from the bucket's 8 lanes (all lanes of the wave still run
    // here, so every shuffle source is active)
    const bool deep_now = d >= B.dwave_tiny;
    if (__ballot(deep_now)) {
      uint32_t cnt = 1, r = 0;  // this lane, then the others of its bucket
      const uint32_t hc = kW == 8 ? g8_mirror(cls) : 0u;
      auto member = [&](uint32_t src, uint32_t cj) {
        if (cj == cls) {
          cnt++;
          r += src < lane;
        }
      };
      member(lane ^ 1u, g8_xor<1>(cls, hc));
      if constexpr (kW == 8) {
        member(lane ^ 2u, g8_xor<2>(cls, hc));
        member(lane ^ 3u, g8_xor<3>(cls, hc));
        member(lane ^ 4u, g8_xor<4>(cls, hc));
        member(lane ^ 5u, g8_xor<5>(cls, hc));
        member(lane ^ 6u, g8_xor<6>(cls, hc));
        member(lane ^ 7u, g8_xor<7>(cls, hc));
      }
      if (deep_now && !done) B.sa[s0 + pos + r] = v;
      if constexpr (kW == 2) {  // a pair bucket is one deep group: its own slot, no atomics
        if (deep_now && !done && r == 0) O.tdeep[bi] = Grp{s0 + pos, cnt, unit, grp_flags(0u, d, 1u)};
      } else {  // at most 4 deep groups per bucket: the bucket's own slots
        const bool lead = deep_now && !done && r == 0;
        const uint64_t bl = __ballot(lead) & (0xffull << (lane & ~7u));
        if (lead) O.dslot[(size_t)bi * 4 + __popcll(bl & lanemask_lt())] = Grp{s0 + pos, cnt, unit, grp_flags(0u, d, 1u)};
        if (deep_now && el == 0 && bi < n_tiny) O.dnum[bi] = (uint32_t)__popcll(bl);
      }
      if (deep_now) break;
    }
    if constexpr (kW == 2) {
      // a pair still tied after a step (long repeats) skips its common prefix 64 characters
      // at a time: both members' next 64 characters, exchanged with the partner lane by DPP,
      // compared word by word; the depth moves to the first differing word (the next 16-
      // character step then orders the pair there)
      bool skipping = !done && pos_step;
      for (;;) {
        const uint32_t q = skipping ? cyc_pos(v, d, U.len) : 0u;
        const bool wrap = skipping && q + 68 > U.len;
        skipping = skipping && !wrap && d < B.dwave_tiny;
        // both members of the pair skip or neither (a member near the unit end stops both)
        // (the exchange runs on every lane: under `skipping &&` it would read disabled lanes)
        const int partner = __builtin_amdgcn_mov_dpp(skipping ? 1 : 0, 0xB1, 0xF, 0xF, false);
        skipping = skipping && partner != 0;
        if (__ballot(skipping) == 0) break;
        uint32_t raw[17], w[16];
        text_raw<16>(t + q, raw);
        text_words_of<16>(t + q, raw, w);
        uint32_t diff = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
          const uint32_t o = (uint32_t)__builtin_amdgcn_mov_dpp((int)w[j], 0xB1, 0xF, 0xF, false);  // lane ^ 1
          diff |= (o != w[j] ? 1u : 0u) << j;
        }
        if (skipping) {
          if (diff == 0) {
            d += 64;
          } else {
            d += 4u * (uint32_t)__builtin_ctz(diff);
            skipping = false;
          }
        }
      }
      pos_step = true;
      if (__ballot(!done && d >= B.dwave_tiny)) continue;  // to the deep branch above
    }
    if constexpr (kW == 8) {
      // a bucket whose live members are all still tied with their classes after a step skips
      // the common prefix of all of them, 64 characters at a time: every live member compares
      // its next 64 characters with its class's first member (ds_bpermute), and the bucket
      // advances to the first word where any member differs.  The depth stays one per bucket
      // (its lanes take the deep branch together), so every DPP source stays active.
      auto b_or = [](uint32_t x) {
        x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // quad xor 1
        x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // quad xor 2
        return x | g8_mirror(x);                                                 // other quad
      };
      auto b_min = [](uint32_t x) {
        x = min(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false));
        x = min(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false));
        return min(x, g8_mirror(x));
      };
      bool skipping = pos_step;
      for (;;) {
        const bool live = !done;
        const uint32_t q = live ? cyc_pos(v, d, U.len) : 0u;
        const uint32_t f = b_or((live ? 1u : 0u) | ((live && q + 68 > U.len) ? 2u : 0u));
        skipping = skipping && f == 1u && d < B.dwave_tiny;  // some member live, none wraps
        if (__ballot(skipping) == 0) break;
        uint32_t raw[17], w[16];
        text_raw<16>(t + q, raw);
        text_words_of<16>(t + q, raw, w);
        const int src = (int)(live ? cls : lane);
        uint32_t diff = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
          const uint32_t o = (uint32_t)__shfl((int)w[j], src, 64);  // the class's first member
          diff |= (o != w[j] ? 1u : 0u) << j;
        }
        const uint32_t fd = b_min(diff ? (uint32_t)__builtin_ctz(diff) : 16u);
        if (skipping) {
          if (fd == 16u) {
            d += 64;
          } else {
            d += 4u * fd;
            skipping = false;
          }
        }
      }
      pos_step = true;
      if (__ballot(!done && d >= B.dwave_tiny)) continue;  // to the deep branch above
    }
    uint32_t k[4] = {0u, 0u, 0u, 0u};
    if (!done) text_key16(t, U.len, cyc_pos(v, d, U.len), k);
    const uint64_t khi = ((uint64_t)k[0] << 32) | k[1], klo = ((uint64_t)k[2] << 32) | k[3];
    // compare with the other 7 lanes of the group (DPP exchanges; this lane counts as equal)
    uint32_t lt = 0, eq = 1, rep = lane;
    {
      uint32_t hc = 0, h0 = 0, h1 = 0, h2 = 0, h3 = 0;
      if constexpr (kW == 8) {
        hc = g8_mirror(cls);
        h0 = g8_mirror(k[0]);
        h1 = g8_mirror(k[1]);
        h2 = g8_mirror(k[2]);
        h3 = g8_mirror(k[3]);
      }
      auto member = [&](uint32_t src, uint32_t cj, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
        const uint64_t hj = ((uint64_t)a0 << 32) | a1, lj = ((uint64_t)a2 << 32) | a3;
        if (cj == cls) {
          lt += (hj < khi) || (hj == khi && lj < klo);
          if (hj == khi && lj == klo) {
            rep = min(rep, src);
            eq++;
          }
        }
      };
#define BZG_G8(M) member(lane ^ (uint32_t)(M), g8_xor<M>(cls, hc), g8_xor<M>(k[0], h0), g8_xor<M>(k[1], h1), \
                         g8_xor<M>(k[2], h2), g8_xor<M>(k[3], h3))
      BZG_G8(1);
      if constexpr (kW == 8) {
        BZG_G8(2);
        BZG_G8(3);
        BZG_G8(4);
        BZG_G8(5);
        BZG_G8(6);
        BZG_G8(7);
      }
#undef BZG_G8
    }
    if (!done) {
      pos += lt;
      cls = rep;
      if (eq == 1) {
        done = true;
        cls = 0xffffffffu;
        const uint32_t slot = s0 + pos;
        B.sa[slot] = v;
        const uint32_t r = slot - U.sbase;
        if (U.k == 1) O.bwt[U.toff + r] = lastc;
        if (v == 0) O.rank0[unit] = r;
      }
    }
    d += 16;
  }
}

// The deep pairs of a k_tiny<2> launch (entries of size 0: none) appended to the deep list,
// one atomic per workgroup of 4096 entries (a single-address atomic per wave, 1.5 M of them
// for long repeats, serialised to tens of ms).
constexpr uint32_t kCompactPer = 16;
__device__ __forceinline__ void deep_compact1(const Grp* __restrict__ in, uint32_t n, Grp* __restrict__ out,
                                              uint32_t* __restrict__ cnt, uint32_t wg) {
  __shared__ uint32_t sh[kT / 64];
  __shared__ uint32_t base;
  const uint32_t i0 = (wg * kT + threadIdx.x) * kCompactPer;
  Grp g[kCompactPer];
  uint32_t k = 0;
#pragma unroll
  for (uint32_t j = 0; j < kCompactPer; j++) {
    g[j] = i0 + j < n ? in[i0 + j] : Grp{0, 0, 0, 0};
    k += g[j].size ? 1u : 0u;
  }
  uint32_t tot;
  const uint32_t ex = block_incl_sum(k, sh, &tot) - k;
  if (threadIdx.x == 0) base = tot ? atomicAdd(cnt, tot) : 0u;
  __syncthreads();
  uint32_t p = base + ex;
#pragma unroll
  for (uint32_t j = 0; j < kCompactPer; j++)
    if (g[j].size) out[p++] = g[j];
}

// Deep groups in per-item slots ([i * m, i * m + num[i])) appended to the deep list, one
// atomic per workgroup.
__device__ __forceinline__ void deep_compact2(const Grp* __restrict__ slot, const uint32_t* __restrict__ num,
                                              uint32_t n, uint32_t m, Grp* __restrict__ out,
                                              uint32_t* __restrict__ cnt, uint32_t wg) {
  __shared__ uint32_t sh[kT / 64];
  __shared__ uint32_t base;
  const uint32_t i0 = (wg * kT + threadIdx.x) * kCompactPer;
  uint32_t c[kCompactPer], k = 0;
#pragma unroll
  for (uint32_t j = 0; j < kCompactPer; j++) {
    c[j] = i0 + j < n ? num[i0 + j] : 0u;
    k += c[j];
  }
  uint32_t tot;
  const uint32_t ex = block_incl_sum(k, sh, &tot) - k;
  if (threadIdx.x == 0) base = tot ? atomicAdd(cnt, tot) : 0u;
  __syncthreads();
  uint32_t p = base + ex;
  for (uint32_t j = 0; j < kCompactPer; j++)
    for (uint32_t x = 0; x < c[j]; x++) out[p++] = slot[(size_t)(i0 + j) * m + x];
}
// The deep groups of one S2 iteration's small classes in one launch: the pair buckets'
// slots (entries of size 0: none; DeepSrc::slot null) and the per-item slots of k_tiny<8> and
// classes 9..32, each source taking its own range of workgroups.
struct DeepSrc {
  const Grp* slot;       // per-item slots [i * m, i * m + num[i]); null: `in` (size 0 = none)
  const Grp* in;
  const uint32_t* num;
  uint32_t n, m, wg0;    // items, slots per item, first workgroup
};
struct DeepSrcs {
  DeepSrc s[4];
  uint32_t ns;
};
__global__ void __launch_bounds__(kT) k_deep_compact_all(DeepSrcs D, Grp* __restrict__ out, uint32_t* __restrict__ cnt) {
  int k = 0;
  while (k + 1 < (int)D.ns && blockIdx.x >= D.s[k + 1].wg0) k++;
  const DeepSrc& S = D.s[k];
  if (S.slot) deep_compact2(S.slot, S.num, S.n, S.m, out, cnt, blockIdx.x - S.wg0);
  else deep_compact1(S.in, S.n, out, cnt, blockIdx.x - S.wg0);
}

// ---- buckets of 9..256 rotations: one segment of kSeg lanes x kPer registers per bucket
// (64 / kSeg buckets per wave).  Element (lane, r) sits at position p = (lane % kSeg) * kPer
// + r of its segment.  Sort key: (run start, 8 characters, element index); pads sort last.
// Round 1 sorts by the first 7 characters after the bucket's depth; every later round
// re-keys only the runs still tied, 6 characters deeper, and re-sorts (positions of unique
// elements never move since their run start is their own position).
// One 64-bit key, so a compare-exchange is one compare and two selects:
//   round 1:  7 characters : 56 | element index : 8
//   later:    run start : 8 | 6 characters : 48 | element index : 8
// Pads are all ones.  No valid key is: the RLE1 output never holds 8 (cyclically) consecutive
// 0xff bytes, so 7 characters of 0xff carry an index below 0xff in a segment with pads (a
// padded segment has fewer than 256 elements); later rounds give valid run starts < 0xff
// there as well, and a run start 0xff would be a singleton, whose key is (position, 0).
using BsortKey = uint64_t;
constexpr BsortKey kPadKey = ~0ull;

// Key layout by elements per wave kE: up to 256 elements, an 8-bit element index under 7
// characters (first round) or an 8-bit run start, 6 characters and the index (later rounds);
// 512 elements (class 257..512), 9-bit indices and run starts with 6 / 5 characters.
template <int kE>
struct KeyFmt {
  static constexpr int kIb = kE > 256 ? 9 : 8;  // index / run-start bits
  static constexpr int kC1 = kE > 256 ? 6 : 7;  // characters of a first-round key
  static constexpr int kC2 = kE > 256 ? 5 : 6;  // characters of a later-round key
  static_assert(kE <= 512, "keys index at most 512 elements");
};
template <int kE = 256>
__device__ __forceinline__ BsortKey make_key1(uint32_t hi, uint32_t lo, uint32_t idx) {
  constexpr int kDrop = 64 - 8 * KeyFmt<kE>::kC1;  // low bits below the kept characters
  return ((((uint64_t)hi << 32) | lo) & ~((1ull << kDrop) - 1ull)) | idx;
}
template <int kE = 256>
__device__ __forceinline__ BsortKey make_key2(uint32_t rs, uint32_t hi, uint32_t lo, uint32_t idx) {
  constexpr int kIb = KeyFmt<kE>::kIb, kCb = 8 * KeyFmt<kE>::kC2;
  return ((uint64_t)rs << (64 - kIb)) | (((((uint64_t)hi << 32) | lo) >> (64 - kCb)) << (64 - kIb - kCb)) | idx;
}
__device__ __forceinline__ bool key_valid(BsortKey k) { return k != kPadKey; }
template <int kE = 256>
__device__ __forceinline__ uint32_t key_idx(BsortKey k) { return (uint32_t)k & ((1u << KeyFmt<kE>::kIb) - 1u); }
// same run start and characters (index ignored)
template <int kE = 256>
__device__ __forceinline__ bool key_tied(BsortKey a, BsortKey b) { return (a >> KeyFmt<kE>::kIb) == (b >> KeyFmt<kE>::kIb); }
__device__ __forceinline__ bool key_less(BsortKey a, BsortKey b) { return a < b; }



// x from lane ^ J (J < 64): DPP quad permutes for 1 and 2, ds_swizzle within 32 lanes,
// ds_bpermute across (DPP / permlane forms for 4..32 measured no faster: the issue stall of the
// network is its dependency chain, profiles/r04_ab_xor_dpp.txt).
__device__ __forceinline__ bool lane_in(uint64_t mask) { return __builtin_amdgcn_inverse_ballot_w64(mask); }
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t x) {
  if constexpr (J == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
  } else if constexpr (J == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
  } else if constexpr (J < 32) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (J << 10) | 0x1F);
  } else {
    return (uint32_t)__shfl_xor((int)x, J, 64);
  }
}

// Direction masks of the bitonic network.  Element r of lane l sits at segment position
// p = (l % kSeg) * kPer + r; at merge size kK and distance kJ it keeps the smaller key of its
// pair iff ((p & kJ) == 0) == ((p & kK) == 0).  These are compile-time wave masks, turned into
// lane conditions by inverse ballot (the mask is the VCC operand: no per-lane arithmetic, no
// live SGPR pairs to spill).
template <int kSeg, int kPer>
constexpr uint64_t keep_min_mask(int kK, int kJ, int r) {
  uint64_t m = 0;
  for (int l = 0; l < 64; l++) {
    const int p = (l % kSeg) * kPer + r;
    if (((p & kJ) == 0) == ((p & kK) == 0)) m |= 1ull << l;
  }
  return m;
}
template <int kSeg, int kPer>
constexpr uint64_t ascending_mask(int kK, int r) {  // lanes whose position p has (p & kK) == 0
  uint64_t m = 0;
  for (int l = 0; l < 64; l++)
    if ((((l % kSeg) * kPer + r) & kK) == 0) m |= 1ull << l;
  return m;
}

template <int kSeg, int kPer, int kK, int kJ>
__device__ __forceinline__ void bitonic_stage(BsortKey (&K)[kPer]) {
  if constexpr (kJ < kPer) {  // partner in another register of this lane
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      const int r2 = r ^ kJ;
      if (r2 > r) {
        // keys are distinct but for pads (equal; swapping them is harmless): one compare
        const bool sw = key_less(K[r2], K[r]) == lane_in(ascending_mask<kSeg, kPer>(kK, r));
        const BsortKey x = K[r], y = K[r2];
        K[r] = sw ? y : x;
        K[r2] = sw ? x : y;
      }
    }
  } else {  // partner lane l ^ (kJ / kPer), same register
    constexpr int jl = kJ / kPer;
    constexpr uint64_t keep = keep_min_mask<kSeg, kPer>(kK, kJ, 0);
    BsortKey o[kPer];
#pragma unroll
    for (int r = 0; r < kPer; r++)
      o[r] = ((uint64_t)xor_lane<jl>((uint32_t)(K[r] >> 32)) << 32) | xor_lane<jl>((uint32_t)K[r]);
#pragma unroll
    for (int r = 0; r < kPer; r++)
      if (lane_in(keep) == key_less(o[r], K[r])) K[r] = o[r];
  }
}
template <int kSeg, int kPer, int kK, int kJ>
__device__ __forceinline__ void bitonic_merge(BsortKey (&K)[kPer]) {
  if constexpr (kJ >= 1) {
    bitonic_stage<kSeg, kPer, kK, kJ>(K);
    bitonic_merge<kSeg, kPer, kK, kJ / 2>(K);
  }
}
template <int kSeg, int kPer, int kK = 2>
__device__ __forceinline__ void bitonic(BsortKey (&K)[kPer]) {
  if constexpr (kK <= kSeg * kPer) {
    bitonic_merge<kSeg, kPer, kK, kK / 2>(K);
    bitonic<kSeg, kPer, kK * 2>(K);
  }
}

// Later rounds of the one-group-per-wave classes only reorder inside the tied runs (keys
// of different runs already differ in their run-start byte), and those runs are short: an
// odd-even transposition sort over the whole segment needs as many steps as the longest run,
// a handful of compare-exchanges with the neighbouring position each, against a full bitonic
// network (21..36 stages).  Positions p = lane * kPer + r; kSeg = 64 (no segment edges).
// Every class gathers 16 characters in its first round (the second round's keys come from LDS
// instead of a second dependent gather).  Rounds after the first whose longest tied run is at
// most kOetsMax use odd-even transposition steps instead of the bitonic network.
constexpr uint32_t kOetsMax = 16;
__device__ __forceinline__ void key_ce(BsortKey& a, BsortKey& b) {
  const bool sw = key_less(b, a);
  const BsortKey x = a, y = b;
  a = sw ? y : x;
  b = sw ? x : y;
}
// Neighbour exchanges and segment scans by DPP (one VALU operation each, no LDS round trip):
// wave_shr:1 / wave_shl:1 move a value one lane up / down (the lane without a source gets 0).
__device__ __forceinline__ uint32_t dpp_up1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false);  // wave_shr:1
}
__device__ __forceinline__ uint32_t dpp_down1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, false);  // wave_shl:1
}
// Inclusive max over the lanes of each kSeg-lane segment (kSeg = 16, 32, 64), up to this lane:
// row_shr 1, 2, 4, 8 inside rows of 16, then row_bcast15 / row_bcast31 across rows.
template <int kSeg>
__device__ __forceinline__ uint32_t seg_incl_max(uint32_t x) {
  static_assert(kSeg == 16 || kSeg == 32 || kSeg == 64, "segments of whole DPP rows");
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));  // row_shr:1
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));  // row_shr:2
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));  // row_shr:4
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));  // row_shr:8
  if constexpr (kSeg >= 32) x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));  // row_bcast15
  if constexpr (kSeg >= 64) x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));  // row_bcast31
  return x;
}
// The same as an inclusive sum over the whole wave.
__device__ __forceinline__ uint32_t wave_incl_sum_dpp(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast31
  return x;
}
__device__ __forceinline__ BsortKey key_shfl_down1(BsortKey k) {
  return ((uint64_t)dpp_down1((uint32_t)(k >> 32)) << 32) | dpp_down1((uint32_t)k);
}
__device__ __forceinline__ BsortKey key_shfl_up1(BsortKey k) {
  return ((uint64_t)dpp_up1((uint32_t)(k >> 32)) << 32) | dpp_up1((uint32_t)k);
}
template <int kSeg, int kPer>
__device__ __forceinline__ void oets(BsortKey (&K)[kPer], uint32_t steps) {
  const uint32_t lane = __lane_id(), sl = lane % kSeg;
  for (uint32_t s = 0; s < steps; s++) {
    const uint32_t par = s & 1u;
    if constexpr (kPer == 1) {
      // pairs (lane, lane + 1) with lane % 2 == par
      const BsortKey nx = key_shfl_down1(K[0]), pv = key_shfl_up1(K[0]);
      const bool left = (lane & 1u) == par;
      if (left && sl < kSeg - 1) K[0] = key_less(nx, K[0]) ? nx : K[0];
      if (!left && sl > 0) K[0] = key_less(K[0], pv) ? pv : K[0];
    } else {
      static_assert((kPer & 1) == 0, "even registers per lane");
      if (par == 0) {
#pragma unroll
        for (int r = 0; r + 1 < kPer; r += 2) key_ce(K[r], K[r + 1]);
      } else {
#pragma unroll
        for (int r = 1; r + 1 < kPer; r += 2) key_ce(K[r], K[r + 1]);
        const BsortKey nx = key_shfl_down1(K[0]), pv = key_shfl_up1(K[kPer - 1]);
        if (sl < kSeg - 1 && key_less(nx, K[kPer - 1])) K[kPer - 1] = nx;
        if (sl > 0 && key_less(K[0], pv)) K[0] = pv;
      }
    }
  }
}

// Later rounds of the one-group-per-wave classes with several registers per lane, when the
// tied runs are too long for the transposition sort: if at most 64 elements are still tied,
// they are packed one per lane (in sorted order, through the wave's 64-key LDS scratch X),
// sorted by a 64-key network (21 stages instead of 28 / 36) and put back.  The tied runs keep
// their places (their keys lead with the run start), so the packed order maps back 1:1.
// Returns false (nothing done) when more than 64 are tied.
template <int kPer>
__device__ __forceinline__ bool compact_sort(BsortKey (&K)[kPer], const bool (&done)[kPer], uint64_t* X) {
  uint32_t mine = 0;
#pragma unroll
  for (int r = 0; r < kPer; r++) mine += (key_valid(K[r]) && !done[r]) ? 1u : 0u;
  const uint32_t incl = wave_incl_sum_dpp(mine);
  const uint32_t nt = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  if (nt > 64) return false;
  const uint32_t lane = __lane_id();
  uint32_t ci = incl - mine;
#pragma unroll
  for (int r = 0; r < kPer; r++)
    if (key_valid(K[r]) && !done[r]) X[ci++] = K[r];
  wave_sync();
  BsortKey k1[1] = {lane < nt ? X[lane] : kPadKey};
  wave_sync();
  bitonic<64, 1>(k1);
  X[lane] = k1[0];
  wave_sync();
  ci = incl - mine;
#pragma unroll
  for (int r = 0; r < kPer; r++)
    if (key_valid(K[r]) && !done[r]) K[r] = X[ci++];
  wave_sync();
  return true;
}

// A group whose members are all still tied (one run: boilerplate, long repeats) advances its
// depth by the members' common prefix, 32 characters per step, instead of 6-7 characters per
// sorting round: every member's next 64 characters are compared with those of the first
// member (lane 0, register 0), word by word; the depth moves to the first word where some
// member differs.  Stops at `limit` and where a member's window wraps past the unit end.
constexpr int kS2Early = 2;  // emitting classes: rounds after which runs of at most two are emitted
template <int kPer>
__device__ __forceinline__ uint32_t common_depth(const uint8_t* t, uint32_t len, const uint32_t (&v)[kPer],
                                                 const bool (&live)[kPer], uint32_t depth, uint32_t limit) {
  constexpr int kW = 8;  // words (32 characters) per step; one member at a time keeps few registers live
  while (depth < limit) {
    bool wrap = false;
#pragma unroll
    for (int r = 0; r < kPer; r++) wrap |= live[r] && cyc_pos(v[r], depth, len) + 4 * kW + 4 > len;
    if (__ballot(wrap)) break;
    uint32_t ref[kW], diff = 0;  // bit j: some member differs from the first in word j
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      const uint32_t q = live[r] ? cyc_pos(v[r], depth, len) : 0u;
      uint32_t raw[kW + 1], k[kW];
      text_raw<kW>(t + q, raw);
      text_words_of<kW>(t + q, raw, k);
#pragma unroll
      for (int j = 0; j < kW; j++) {
        if (r == 0) ref[j] = (uint32_t)__builtin_amdgcn_readlane((int)k[j], 0);
        if (__ballot(live[r] && k[j] != ref[j])) diff |= 1u << j;
      }
    }
    if (diff == 0) {
      depth += 4 * kW;
    } else {
      depth += 4u * (uint32_t)__builtin_ctz(diff);
      break;
    }
  }
  return depth;
}

// Runs still tied after kRounds bitonic rounds (few rotations, often long repeats) are
// finished in place: every tied rotation ranks itself among the members of its run that are
// still tied with it (same class, named by the lowest position of the class) on the next 16
// characters per step; positions do not move any more, the final slot is run start + rank.


template <int kSeg, int kPer, bool kBatch>
__device__ void bsort_tail(const SortBufs& B, const SortOut& O, const Grp& g, uint32_t bi, const Unit& U, uint32_t depth,
                           const BsortKey (&K)[kPer], const bool (&done)[kPer], const uint32_t (&rsn)[kPer],
                           const uint32_t* Lv, uint32_t* Lk, uint4* TK, uint32_t* TC) {
  constexpr int kN = kSeg * kPer;
  const uint32_t lane = __lane_id(), sl = lane % kSeg, sb = (lane / kSeg) * kN;
  const uint8_t* t = B.text + U.toff;
  bool live[kPer];
  uint32_t v[kPer], pos[kPer], cls[kPer], rlen[kPer];
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    live[r] = !done[r] && key_valid(K[r]);
    v[r] = live[r] ? Lv[key_idx(K[r])] : 0u;
    pos[r] = rsn[r];
    cls[r] = rsn[r];
    Lk[lane * kPer + r] = 0;
  }
  wave_sync();
#pragma unroll
  for (int r = 0; r < kPer; r++)
    if (live[r]) atomicAdd(&Lk[sb + rsn[r]], 1u);
  wave_sync();
#pragma unroll
  for (int r = 0; r < kPer; r++) rlen[r] = live[r] ? Lk[sb + rsn[r]] : 0u;
  for (;;) {
    bool any = false;
#pragma unroll
    for (int r = 0; r < kPer; r++) any |= live[r];
    if (__ballot(any) == 0) break;
    const bool deep = depth >= B.dwave;
    if constexpr (kBatch) {
      uint32_t raw[kPer][5], qq[kPer];
#pragma unroll
      for (int r = 0; r < kPer; r++) {
        qq[r] = live[r] ? cyc_pos(v[r], depth, U.len) : 0u;
        text_raw<4>(t + qq[r], raw[r]);
      }
#pragma unroll
      for (int r = 0; r < kPer; r++) {
        const uint32_t wp = sb + sl * kPer + r;
        uint32_t k[4];
        text_words_of<4>(t + qq[r], raw[r], k);
        if (live[r] && qq[r] + 16 > U.len) text_words_wrap<4>(t, U.len, qq[r], k);
        TK[wp] = make_uint4(k[0], k[1], k[2], k[3]);
        TC[wp] = live[r] ? cls[r] : 0xffffffffu;
      }
    } else {
#pragma unroll
      for (int r = 0; r < kPer; r++) {
        const uint32_t wp = sb + sl * kPer + r;
        uint32_t k[4] = {0u, 0u, 0u, 0u};
        if (live[r] && !deep) text_key16(t, U.len, cyc_pos(v[r], depth, U.len), k);
        TK[wp] = make_uint4(k[0], k[1], k[2], k[3]);
        TC[wp] = live[r] ? cls[r] : 0xffffffffu;
      }
    }
    wave_sync();
    if (deep) {  // still tied after B.dwave characters: leave to the doubling fallback
      static_assert(kPer == 1, "one rotation per lane: a segment's deep groups are counted by ballot");
      // (all lanes of a segment take this branch together: depth is the segment's)
      const uint32_t p = sl;
      uint32_t rank = 0, cnt = 0;
      if (live[0]) {
        for (uint32_t q = rsn[0]; q < rsn[0] + rlen[0]; q++)
          if (TC[sb + q] == cls[0]) {
            cnt++;
            rank += q < p;
          }
        B.sa[g.start + pos[0] + rank] = v[0];
      }
      // the segment's deep groups go to its own slots (a single-address atomic per wave
      // serialises when long repeats make millions of them)
      const bool lead = live[0] && rank == 0;
      const uint64_t seg = (kSeg == 64 ? ~0ull : ((1ull << kSeg) - 1ull)) << (lane - sl);
      const uint64_t bl = __ballot(lead) & seg;
      if (lead) O.dslot[(size_t)bi * O.dm + __popcll(bl & lanemask_lt())] = Grp{g.start + pos[0], cnt, g.unit, grp_flags(0u, depth, 2u)};
      if (sl == 0) O.dnum[bi] = (uint32_t)__popcll(bl);
      break;
    }
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      if (!live[r]) continue;
      const uint4 me = TK[sb + sl * kPer + r];
      const uint64_t mh = ((uint64_t)me.x << 32) | me.y, ml = ((uint64_t)me.z << 32) | me.w;
      uint32_t lt = 0, eq = 0, rep = 0xffffffffu;
      for (uint32_t q = rsn[r]; q < rsn[r] + rlen[r]; q++) {
        if (TC[sb + q] != cls[r]) continue;
        const uint4 o = TK[sb + q];
        const uint64_t oh = ((uint64_t)o.x << 32) | o.y, ol = ((uint64_t)o.z << 32) | o.w;
        lt += (oh < mh) || (oh == mh && ol < ml);
        if (oh == mh && ol == ml) {
          if (rep == 0xffffffffu) rep = q;
          eq++;
        }
      }
      pos[r] += lt;
      cls[r] = rep;
      if (eq == 1) {
        live[r] = false;
        const uint32_t slot = g.start + pos[r];
        B.sa[slot] = v[r];
        const uint32_t rr = slot - U.sbase;
        if (U.k == 1) O.bwt[U.toff + rr] = t[v[r] == 0 ? U.len - 1 : v[r] - 1];
        if (v[r] == 0) O.rank0[g.unit] = rr;
      }
    }
    wave_sync();
    depth += 16;
  }
}


// S2 run emission (classes with one group per wave): after kRounds rounds the runs still tied
// are left as new groups.  Their rotations are stored at their slots (primary SA) and each run
// becomes a record (depth:13 | run start:9 | size:10) in the group's own part of `rec` (from
// half its first slot; a group of m has at most m / 2 runs), with per-class counts
// ccnt[c * total + gbase + list index] for the class-major scan.  k_s2_emit builds the lists.
__device__ __forceinline__ uint32_t s2_rec(uint32_t depth, uint32_t rs, uint32_t size) {
  return (depth << 19) | (rs << 10) | size;
}
struct S2Emit {
  uint32_t* rec;
  uint32_t* ccnt;
  uint32_t total, gbase;
};

template <int kSeg, int kPer, int kRounds, bool kBatch, bool kEmit = false>
__global__ void __launch_bounds__(kT) BZG_SGPR_LIMIT k_bsort(const Grp* __restrict__ L, uint32_t nL, SortBufs B, SortOut O,
                                              S2Emit E = S2Emit{}) {
  constexpr int kBPW = 64 / kSeg;
  constexpr int kE = 64 * kPer;  // elements per wave
  // the rank-counting tail (TK, TC, Lk) only exists without emission: the emitting classes
  // hand runs still tied at B.dwave to the doubling fallback directly, so they need little LDS
  // and run at full occupancy
  constexpr int kTE = kEmit ? 1 : kE;
  __shared__ uint32_t Lv[kT / 64][kE];
  __shared__ uint8_t Lc[kT / 64][kE];
  __shared__ uint32_t Lk[kT / 64][kEmit ? 8 : kE];
  __shared__ uint4 TK[kT / 64][kTE];
  __shared__ uint32_t TC[kT / 64][kTE];
  constexpr bool kPre = true;
  __shared__ uint64_t Lx[kT / 64][kPre ? kE : 1];  // characters depth + 7 .. + 14 (second-round keys)
  const uint32_t w = threadIdx.x >> 6, lane = __lane_id();
  const uint32_t sl = lane % kSeg;
  const uint32_t bi = (s2_wg() * (kT / 64) + w) * kBPW + lane / kSeg;
  const bool has = bi < nL;
  if (__ballot(has) == 0) return;
  Grp g{0, 0, 0, 0};
  if (has) g = L[bi];
  if constexpr (!kEmit) {
    if (has && sl == 0) O.dnum[bi] = 0;  // (bsort_tail counts the group's deep groups here)
  }
  Unit U{0, 1, 0, 1};
  if (has) U = B.units[g.unit];
  const uint8_t* t = B.text + U.toff;
  const uint32_t m = g.size;
  uint32_t depth = grp_depth(g);
  const uint32_t* src = (g.flags & kGrpAlt) ? B.sa2 : B.sa;
  BsortKey K[kPer];
  uint32_t vq[kPer];
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    const uint32_t p = sl * kPer + r;
    vq[r] = p < m ? ((g.flags & kGrpIdent) ? p : src[g.start + p]) : 0u;
  }
  if constexpr (kPre) {
    // one round trip for two rounds: 16 characters per rotation, the 8 after the first 7
    // kept in LDS for the second round's keys (almost every wave of these classes has one)
    // (4 aligned words hold at least 13 characters from any start: the kC1 + kC2 the two rounds
    // use; a fifth word per rotation held class 257..512 at 4 waves per SIMD)
    uint32_t raw[kPer][4], cq[kPer];
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      cq[r] = cyc_pos(vq[r], depth, U.len);
      text_raw<3>(t + cq[r], raw[r]);
      cq[r] |= (uint32_t)t[vq[r] == 0 ? U.len - 1 : vq[r] - 1] << 24;
    }
    static_assert(KeyFmt<kE>::kC1 + KeyFmt<kE>::kC2 <= 13, "four aligned words per rotation");
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      const uint32_t p = sl * kPer + r, idx = lane * kPer + r;
      const bool valid = p < m;
      const uint32_t q = cq[r] & 0xffffffu;
      uint32_t k4[4];
      {
        uint32_t k3[3];
        text_words_of<3>(t + q, raw[r], k3);
        k4[0] = k3[0], k4[1] = k3[1], k4[2] = k3[2];
        // characters 12 .. 15 - (start & 3) of the last word (the rest are not used)
        k4[3] = __builtin_bswap32(__builtin_amdgcn_alignbyte(0u, raw[r][3], (uint32_t)((uintptr_t)(t + q) & 3u)));
      }
      if (valid && q + 13 > U.len) text_words_wrap<4>(t, U.len, q, k4);
      Lv[w][idx] = vq[r];
      Lc[w][idx] = (uint8_t)(cq[r] >> 24);
      constexpr uint32_t kSh = 8 * (KeyFmt<kE>::kC1 - 4);  // the 8 characters after the first kC1
      Lx[w][idx] = ((uint64_t)((k4[1] << kSh) | (k4[2] >> (32 - kSh))) << 32) | ((k4[2] << kSh) | (k4[3] >> (32 - kSh)));
      K[r] = valid ? make_key1<kE>(k4[0], k4[1], idx) : kPadKey;
    }
  } else if constexpr (kBatch) {
    // all loads issued before any is used (3 aligned words and the BWT byte per rotation);
    // keys that wrap past the unit end are rebuilt afterwards
    uint32_t raw[kPer][3], cq[kPer];
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      cq[r] = cyc_pos(vq[r], depth, U.len);
      text_raw<2>(t + cq[r], raw[r]);
      cq[r] |= (uint32_t)t[vq[r] == 0 ? U.len - 1 : vq[r] - 1] << 24;
    }
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      const uint32_t p = sl * kPer + r, idx = lane * kPer + r;
      const bool valid = p < m;
      const uint32_t q = cq[r] & 0xffffffu;
      uint32_t k2[2];
      text_words_of<2>(t + q, raw[r], k2);
      if (valid && q + 8 > U.len) text_words_wrap<2>(t, U.len, q, k2);
      Lv[w][idx] = vq[r];
      Lc[w][idx] = (uint8_t)(cq[r] >> 24);
      K[r] = valid ? make_key1<kE>(k2[0], k2[1], idx) : kPadKey;
    }
  } else {
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      const uint32_t p = sl * kPer + r, idx = lane * kPer + r;
      const bool valid = p < m;
      uint32_t hi = 0xffffffffu, lo = 0xffffffffu;
      uint8_t c = 0;
      if (valid) {
        text_key8(t, U.len, cyc_pos(vq[r], depth, U.len), hi, lo);
        c = t[vq[r] == 0 ? U.len - 1 : vq[r] - 1];
      }
      Lv[w][idx] = vq[r];
      Lc[w][idx] = c;
      K[r] = valid ? make_key1<kE>(hi, lo, idx) : kPadKey;
    }
  }
  bool done[kPer];
#pragma unroll
  for (int r = 0; r < kPer; r++) done[r] = false;
  int round = 0;
  bool skipped = false;  // common_depth moved the depth: the second-round keys in Lx are stale
  uint32_t maxrun = 0;  // longest tied run of the previous round (kSeg = 64)
  // BZG_DEBUG: waves entering each round, per class (dbg[8 + 8 * class + round]; round 7:
  // the rank-counting tail)
  constexpr int kDbgCls = kSeg * kPer == 16 ? 1 : kSeg * kPer == 32 ? 2 : kSeg * kPer == 64 ? 3 : kSeg * kPer == 128 ? 4
                         : kSeg * kPer == 256 ? 5 : 6;
  for (;;) {
    if (O.dbg && lane == 0) atomicAdd(&O.dbg[8 + 8 * kDbgCls + min(round, 6)], 1ull);
    if (O.dbg && round > 0 && kDbgCls >= 3) {  // later rounds: longest tied run and tied elements
      uint32_t nt = 0;
#pragma unroll
      for (int r = 0; r < kPer; r++) nt += (key_valid(K[r]) && !done[r]) ? 1u : 0u;
      nt = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(nt), 63);
      auto bk = [](uint32_t x) { return x <= 4 ? 0 : x <= 8 ? 1 : x <= 16 ? 2 : x <= 32 ? 3 : x <= 64 ? 4 : 5; };
      if (lane == 0) {
        atomicAdd(&O.dbg[64 + 16 * (kDbgCls - 3) + bk(maxrun)], 1ull);
        atomicAdd(&O.dbg[64 + 16 * (kDbgCls - 3) + 8 + bk(nt)], 1ull);
      }
    }
    if (round > 0 && maxrun <= kOetsMax)
      oets<kSeg, kPer>(K, maxrun);
    else if (!(kSeg == 64 && kPer > 1 && kPre && round > 0 && compact_sort<kPer>(K, done, Lx[w])))
      bitonic<kSeg, kPer>(K);
    // ties with the previous / next position of the segment (same run start and key)
    bool tp[kPer], tn[kPer];
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      BsortKey q;
      if (r > 0) {
        q = K[r - 1];
      } else {
        q = key_shfl_up1(K[kPer - 1]);
        if (sl == 0) q = ~K[r];  // no previous element
      }
      tp[r] = key_valid(K[r]) && key_tied<kE>(q, K[r]);
    }
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      if (r + 1 < kPer) {
        tn[r] = tp[r + 1];
      } else {
        bool x = dpp_down1(tp[0] ? 1u : 0u) != 0;
        if (sl == kSeg - 1) x = false;
        tn[r] = x;
      }
    }
    // positions (sorted order); new run starts: p if it starts a run, else inherited
    uint32_t rsn[kPer];
    uint32_t mx = 0;
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      const uint32_t p = sl * kPer + r;
      mx = max(mx, tp[r] ? 0u : p);
      rsn[r] = mx;
    }
    uint32_t pre = dpp_up1(seg_incl_max<kSeg>(mx));
    if (sl == 0) pre = 0;
    bool any_tied = false;
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      rsn[r] = max(rsn[r], pre);
      const uint32_t idx = key_idx<kE>(K[r]);
      const bool valid = key_valid(K[r]);
      const bool tied = valid && (tp[r] || tn[r]);
      const uint32_t p = sl * kPer + r;
      if (valid && !tied && !done[r]) {
        // unique: final position
        const uint32_t slot = g.start + p;
        const uint32_t v = Lv[w][idx];
        B.sa[slot] = v;
        const uint32_t rr = slot - U.sbase;
        if (U.k == 1) O.bwt[U.toff + rr] = Lc[w][idx];
        if (v == 0) O.rank0[g.unit] = rr;
      }
      done[r] = valid && !tied;
      any_tied |= tied;
    }
    if (__ballot(any_tied) == 0) {
      if constexpr (kEmit) {  // no records: the group's class counts are 0
        if (lane < (uint32_t)kS2Cls) E.ccnt[(size_t)lane * E.total + E.gbase + bi] = 0u;
      }
      break;
    }
    depth += round == 0 ? KeyFmt<kE>::kC1 : KeyFmt<kE>::kC2;  // tied runs are equal to this depth
    if constexpr (kSeg == 64 && kPer <= 2) {  // (kPer 4: the registers would cost a wave per SIMD)
      bool split = false;  // the group is no longer one run
#pragma unroll
      for (int r = 0; r < kPer; r++) split |= key_valid(K[r]) && (done[r] || rsn[r] != 0);
      if (__ballot(split) == 0 && depth < B.dwave) {
        uint32_t vv[kPer];
        bool live[kPer];
#pragma unroll
        for (int r = 0; r < kPer; r++) {
          live[r] = key_valid(K[r]);
          vv[r] = live[r] ? Lv[w][key_idx<kE>(K[r])] : 0u;
        }
        const uint32_t d2 = common_depth<kPer>(t, U.len, vv, live, depth, B.dwave);
        skipped |= d2 != depth;
        depth = d2;
      }
    }
    {  // longest tied run (next round's network; early emission)
      uint32_t ml = 0;
#pragma unroll
      for (int r = 0; r < kPer; r++)
        if (key_valid(K[r]) && !done[r] && !tn[r]) ml = max(ml, sl * kPer + r - rsn[r] + 1);
      maxrun = (uint32_t)__builtin_amdgcn_readlane((int)seg_incl_max<64>(ml), 63);
    }
    // only pairs still tied after kS2Early rounds (long repeats: the pairs of a copied
    // passage stay tied round after round): emitted now, as the pair lists' 64-character skip
    // (k_tiny<2>) resolves or deepens them far cheaper than further rounds of the whole network
    const bool early = kEmit && round + 1 >= kS2Early && maxrun <= 2;
    if (++round >= kRounds || depth >= B.dwave || early) {
      if constexpr (kEmit) {
        static_assert(kSeg == 64, "one group per wave");
        {
          uint32_t* cc = Lk[w];  // per-class counters, then the record cursor
          if (lane < 8) cc[lane] = 0;
          wave_sync();
#pragma unroll
          for (int r = 0; r < kPer; r++) {
            if (!key_valid(K[r]) || done[r]) continue;
            const uint32_t p = sl * kPer + r;
            B.sa[g.start + p] = Lv[w][key_idx<kE>(K[r])];
            if (!tn[r]) {  // last member of its run
              const uint32_t size = p - rsn[r] + 1;
              if (depth >= B.dwave) {  // still tied after B.dwave characters: doubling fallback
                O.deep[wave_append(O.n_deep, true)] = Grp{g.start + rsn[r], size, g.unit, grp_flags(0u, depth, 2u)};
              } else {
                atomicAdd(&cc[size_cls(size)], 1u);
                E.rec[g.start / 2 + atomicAdd(&cc[7], 1u)] = s2_rec(depth, rsn[r], size);
              }
            }
          }
          wave_sync();
          if (lane < (uint32_t)kS2Cls) E.ccnt[(size_t)lane * E.total + E.gbase + bi] = cc[lane];
          break;
        }
      } else {
        if (O.dbg && lane == 0) atomicAdd(&O.dbg[8 + 8 * kDbgCls + 7], 1ull);
        bsort_tail<kSeg, kPer, kBatch>(B, O, g, bi, U, depth, K, done, rsn, Lv[w], Lk[w], TK[w], TC[w]);
      }
      break;
    }
    // re-key the tied runs 8 characters deeper; unique elements keep their own position as run start
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      const uint32_t idx = key_idx<kE>(K[r]);
      if (!key_valid(K[r])) continue;
      const uint32_t p = sl * kPer + r;
      if (done[r]) {
        K[r] = make_key2<kE>(p, 0, 0, idx);
      } else {
        uint32_t hi, lo;
        if (kPre && round == 1 && !skipped) {
          const uint64_t x = Lx[w][kPre ? idx : 0];
          hi = (uint32_t)(x >> 32);
          lo = (uint32_t)x;
        } else {
          text_key8(t, U.len, cyc_pos(Lv[w][idx], depth, U.len), hi, lo);
        }
        K[r] = make_key2<kE>(rsn[r], hi, lo, idx);
      }
    }
  }
}

// The records of the emitting k_bsort launches into the next class lists.  One thread per
// group g of the concatenated classes 3..6 (gb[k]: index of class 3 + k's first group; gb[4]:
// the total).
struct S2Lists {
  const Grp* cur[4];
  uint32_t gb[5];
};
__global__ void k_s2_emit(S2Lists Ls, const uint32_t* __restrict__ rec, const uint32_t* __restrict__ cscan,
                          uint32_t total, ClsLists N, uint32_t* __restrict__ zero2) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < 2) zero2[g] = 0;  // k_split_pairs' output counters, for the next iteration
  if (g >= total) return;
  uint32_t n = 0, pos[kS2Cls];
#pragma unroll
  for (int c = 0; c < kS2Cls; c++) {
    const uint32_t a = cscan[(size_t)c * total + g], e = cscan[(size_t)c * total + g + 1];
    pos[c] = a - cscan[(size_t)c * total];
    n += e - a;
  }
  if (n == 0) return;
  const int k = g >= Ls.gb[3] ? 3 : g >= Ls.gb[2] ? 2 : g >= Ls.gb[1] ? 1 : 0;
  const Grp gr = Ls.cur[k][g - Ls.gb[k]];
  const uint32_t* gr_rec = rec + gr.start / 2;
  for (uint32_t x = 0; x < n; x++) {
    const uint32_t r = gr_rec[x];
    const uint32_t size = r & 1023u, rs = (r >> 10) & 511u, depth = r >> 19;
    const uint32_t c = size_cls(size);
    uint32_t p = 0;
#pragma unroll
    for (int q = 0; q < kS2Cls; q++)
      if ((uint32_t)q == c) p = pos[q]++;
    N.l[c][p] = Grp{gr.start + rs, size, gr.unit, grp_flags(0u, depth, 0u)};
  }
}


// ---------------------------------------------------------------- S2 lists in block order
// The S1 passes append S2 groups pass after pass, each pass sweeping every block, so a list
// is ~a dozen sparse sweeps: the groups in flight at once would span dozens of blocks, whose
// texts do not fit an XCD's L2 together.  Before S2 the lists are counting-sorted by unit
// (block), so the groups in flight come from one or two blocks (order inside a unit is
// immaterial: every group is sorted on its own slots).
// Lanes of a wave sharing a unit reserve consecutive counts with one atomic per unit.
__device__ __forceinline__ uint32_t unit_reserve(uint32_t* __restrict__ ctr, uint32_t unit, bool act) {
  uint64_t left = __ballot(act);
  uint32_t pos = 0;
  const uint32_t lane = __lane_id();
  while (left) {
    const int leader = __ffsll((unsigned long long)left) - 1;
    const uint32_t lu = (uint32_t)__shfl((int)unit, leader, 64);
    const uint64_t m = __ballot(act && unit == lu) & left;
    uint32_t base = 0;
    if (lane == (uint32_t)leader) base = atomicAdd(&ctr[lu], (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, leader, 64);
    if ((m >> lane) & 1ull) pos = base + (uint32_t)__popcll(m & lanemask_lt());
    left &= ~m;
  }
  return pos;
}

__global__ void k_unit_count(const Grp* __restrict__ L, uint32_t n, uint32_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < n;
  (void)unit_reserve(cnt, act ? L[i].unit : 0u, act);
}

__global__ void k_unit_scatter(const Grp* __restrict__ L, uint32_t n, uint32_t* __restrict__ cursor,
                               Grp* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < n;
  Grp g{0, 0, 0, 0};
  if (act) g = L[i];
  const uint32_t p = unit_reserve(cursor, g.unit, act);
  if (act) out[p] = g;
}

// ---------------------------------------------------------------- fallback glue
__global__ void __launch_bounds__(kT) k_fb_flag(const Grp* __restrict__ D, uint32_t n, uint32_t* __restrict__ uflag,
                                                uint32_t* __restrict__ mind) {
  __shared__ uint32_t wmin[kT / 64];
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t d = 0xffffffffu;
  if (g < n) {
    const Grp gr = D[g];
    if (uflag[gr.unit] == 0) uflag[gr.unit] = 1;  // read first: most lanes find it set
    d = grp_depth(gr);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) d = min(d, (uint32_t)__shfl_xor((int)d, o, 64));
  if (__lane_id() == 0) wmin[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {  // one atomic per workgroup (tens of millions of deep groups)
    uint32_t m = wmin[0];
    for (int w = 1; w < kT / 64; w++) m = min(m, wmin[w]);
    // (read first: the depths are nearly all equal, so almost no workgroup needs the
    // single-address atomic, which costs ~10 ns each across 200 k workgroups)
    if (m != 0xffffffffu && m < __hip_atomic_load(mind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(mind, m);
  }
}

// f(group, member) over the members of groups L[0..n): a lane per group walks a small group
// itself, the wave walks the large ones of its 64 together (deep groups are mostly pairs, so a
// workgroup per group left almost every lane idle).
constexpr uint32_t kLaneGroup = 32;
template <typename F>
__device__ __forceinline__ void for_members(const Grp* __restrict__ L, uint32_t n, F&& f) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  Grp gr{0, 0, 0, 0};
  if (g < n) gr = L[g];
  const bool big = gr.size > kLaneGroup;
  if (!big)
    for (uint32_t e = 0; e < gr.size; e++) f(gr, e);
  uint64_t m = __ballot(big);
  while (m) {
    const int l = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    const Grp G{(uint32_t)__shfl((int)gr.start, l, 64), (uint32_t)__shfl((int)gr.size, l, 64),
                (uint32_t)__shfl((int)gr.unit, l, 64), (uint32_t)__shfl((int)gr.flags, l, 64)};
    for (uint32_t e = __lane_id(); e < G.size; e += 64) f(G, e);
  }
}

// Deep groups whose data is in the alternate buffer move to the primary SA; the doubling
// list gets the groups with their flags reset.
__global__ void __launch_bounds__(kT) k_fb_copy(const Grp* __restrict__ D, uint32_t n, Grp* __restrict__ L0, SortBufs B) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n) {
    const Grp gr = D[g];
    L0[g] = Grp{gr.start, gr.size, gr.unit, 0};
  }
  for_members(D, n, [&](const Grp& gr, uint32_t e) {
    if (gr.flags & kGrpAlt) B.sa[gr.start + e] = B.sa2[gr.start + e];
  });
}

// Members of a deep group take the group's first slot as rank (after k_fb_isa_all).
__global__ void __launch_bounds__(kT) k_fb_group_isa(const Grp* __restrict__ L0, uint32_t n, SortBufs B) {
  for_members(L0, n, [&](const Grp& gr, uint32_t e) {
    B.isa[B.units[gr.unit].sbase + B.sa[gr.start + e]] = gr.start;
  });
}

// ISA of every slot of the listed units from the (complete, primary) SA: every rotation's own
// slot; deep groups' members are overwritten afterwards by k_fb_group_isa.  The ISA stores of a
// unit scatter over its whole range, so all workgroups of unit u run on one XCD (hardware
// workgroup w goes to XCD w % 8): its L2 merges the unit's scattered stores into full lines.
// Grid: 8 * ceil(nu / 8) * chunks workgroups.
__global__ void __launch_bounds__(kT) k_fb_isa_all(const uint32_t* __restrict__ ulist, uint32_t nu, uint32_t chunks,
                                                   const Unit* __restrict__ units, SortBufs B) {
  const uint32_t xcd = blockIdx.x % kNumXcd, rest = blockIdx.x / kNumXcd;
  const uint32_t ui = (rest / chunks) * kNumXcd + xcd, ch = rest % chunks;
  if (ui >= nu) return;
  const Unit U = units[ulist[ui]];
  const uint32_t q = ch * kT + threadIdx.x;
  if (q >= U.len) return;
  const uint32_t v = B.sa[U.sbase + q];
  B.isa[U.sbase + v] = U.sbase + q;
}

// ---------------------------------------------------------------- S3 pairs
// Most deep groups are pairs, made by long repeated passages: rotations a and b = a + d tied
// for >= h0 characters.  Their order is decided at the first position p >= a where
// t[p] != t[p + d].  Consecutive pairs (a, a + d), (a + 1, a + d + 1), ... of one passage
// share that position, so it is looked up once, after the pair at the end of the run:
//   pm[x] = partner of x when x is in a deep pair (~0 otherwise); x links to x + 1 when
//   pm[x + 1] = pm[x] + 1 (both in the unit); E(x) = the first unlinked position >= x;
//   the order of (a, b) is the order of (E, pm[E]), tied for >= h0 characters: compare
//   from E + h0 on (usually one character: the pair after E is tied for < h0).
// Pairs whose comparison runs past kPairScan characters (the run continues into a larger
// group) stay for the doubling.  Positions are unit-local; slots sbase + x.
constexpr uint32_t kRunTile = 4096;  // positions per run-end tile (16 per thread)
constexpr uint32_t kPairShort = 2048;    // characters a run-end pair compares on its own lane
constexpr uint32_t kPairScan = 1u << 20;  // and on a whole wave (k_pair_long), at most

__global__ void __launch_bounds__(kT) k_pm_init(const uint32_t* __restrict__ ulist, uint32_t nu, uint32_t chunks,
                                                const Unit* __restrict__ units, uint32_t* __restrict__ pm) {
  const uint32_t ui = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  if (ui >= nu) return;
  const Unit U = units[ulist[ui]];
  for (uint32_t q = ch * kT * 16 + threadIdx.x; q < min(U.len, (ch + 1) * kT * 16); q += kT) pm[U.sbase + q] = 0xffffffffu;
}

__global__ void __launch_bounds__(kT) k_pair_mark(const Grp* __restrict__ L, uint32_t n, SortBufs B,
                                                  uint32_t* __restrict__ pm) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const Grp gr = L[g];
  if (gr.size != 2) return;
  const uint32_t sb = B.units[gr.unit].sbase;
  const uint32_t a = B.sa[gr.start], b = B.sa[gr.start + 1];
  pm[sb + a] = b;
  pm[sb + b] = a;
}

// Run ends inside each tile of kRunTile positions of the listed units: E[x] (unit-local),
// or ~0 when the run goes on past the tile; tsum[tile] = the tile's first unlinked position
// (~0: none).  Tile (ui, c) has index tbase[ui] + c.
__global__ void __launch_bounds__(kT) k_runend_tile(const uint32_t* __restrict__ ulist, const uint32_t* __restrict__ tbase,
                                                    uint32_t nu, const Unit* __restrict__ units,
                                                    const uint32_t* __restrict__ pm, uint32_t* __restrict__ E,
                                                    uint32_t* __restrict__ tsum) {
  __shared__ uint32_t fb[kT];
  const uint32_t ui = blockIdx.y, c = blockIdx.x;
  if (ui >= nu) return;
  const Unit U = units[ulist[ui]];
  const uint32_t t0 = c * kRunTile;
  if (t0 >= U.len) return;  // (uniform)
  const uint32_t* p = pm + U.sbase;
  const uint32_t x0 = t0 + threadIdx.x * 16;
  uint32_t v[17];
#pragma unroll
  for (int k = 0; k < 17; k++) v[k] = x0 + k < U.len ? p[x0 + k] : 0xffffffffu;
  // x links to x + 1: both in the unit, x paired, and pm[x + 1] = pm[x] + 1 without wrapping
  uint32_t lk = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t x = x0 + k;
    const bool l = x + 1 < U.len && v[k] != 0xffffffffu && v[k] + 1 < U.len && v[k + 1] == v[k] + 1;
    lk |= (l ? 1u : 0u) << k;
  }
  // first unlinked position of this thread's slice (every position past the unit end is one)
  const uint32_t nl = ~lk & 0xffffu;
  fb[threadIdx.x] = nl ? x0 + (uint32_t)__builtin_ctz(nl) : 0xffffffffu;
  __syncthreads();
  // suffix minimum over the threads after this one
  for (uint32_t o = 1; o < kT; o <<= 1) {
    const uint32_t y = threadIdx.x + o < kT ? fb[threadIdx.x + o] : 0xffffffffu;
    __syncthreads();
    fb[threadIdx.x] = min(fb[threadIdx.x], y);
    __syncthreads();
  }
  const uint32_t after = threadIdx.x + 1 < kT ? fb[threadIdx.x + 1] : 0xffffffffu;
  if (threadIdx.x == 0) tsum[tbase[ui] + c] = fb[0];
  uint32_t e = after;
#pragma unroll
  for (int k = 15; k >= 0; k--) {
    const uint32_t x = x0 + k;
    if (!((lk >> k) & 1u)) e = x;
    if (x < U.len && v[k] != 0xffffffffu) E[U.sbase + x] = e;
  }
}

// F[tile] = the first unlinked position at or after the tile's start (walks the following
// tiles of the unit; the unit's last position is always unlinked).
__global__ void k_runend_tiles(const uint32_t* __restrict__ ulist, const uint32_t* __restrict__ tbase, uint32_t nu,
                               const Unit* __restrict__ units, const uint32_t* __restrict__ tsum,
                               uint32_t* __restrict__ F) {
  const uint32_t ui = blockIdx.y, c = blockIdx.x * blockDim.x + threadIdx.x;
  if (ui >= nu) return;
  const uint32_t nt = ceil_div(units[ulist[ui]].len, kRunTile);
  if (c >= nt) return;
  const uint32_t tb = tbase[ui];
  uint32_t k = c;
  while (tsum[tb + k] == 0xffffffffu && k + 1 < nt) k++;
  F[tb + c] = tsum[tb + k];
}

// First mismatch of rotations e and f (tied for >= h0 characters) within `limit` characters
// from character h0: -1 (e first), +1 (f first) or 0 (none found).  16 characters per step.
__device__ int pair_order(const uint8_t* t, uint32_t len, uint32_t e, uint32_t f, uint32_t h0, uint32_t limit) {
  uint32_t qe = cyc_pos(e, h0, len), qf = cyc_pos(f, h0, len);
  for (uint32_t k = 0; k < limit; k += 16) {
    uint32_t xe[4], xf[4];
    if (qe + 16 <= len && qf + 16 <= len) {
      text_key16(t, len, qe, xe);
      text_key16(t, len, qf, xf);
    } else {
      text_words_wrap<4>(t, len, qe, xe);
      text_words_wrap<4>(t, len, qf, xf);
    }
#pragma unroll
    for (int w = 0; w < 4; w++)
      if (xe[w] != xf[w]) return xe[w] < xf[w] ? -1 : 1;
    qe += 16;
    if (qe >= len) qe -= len;
    qf += 16;
    if (qf >= len) qf -= len;
  }
  return 0;
}

// Orders the pair in slots (start, start + 1): lo first.
__device__ __forceinline__ void pair_write(const SortBufs& B, const SortOut& O, const Grp& gr, const Unit& U,
                                           const uint8_t* t, uint32_t lo, uint32_t hi) {
  B.sa[gr.start] = lo;
  B.sa[gr.start + 1] = hi;
  const uint32_t r = gr.start - U.sbase;
  if (U.k == 1) {
    O.bwt[U.toff + r] = t[lo == 0 ? U.len - 1 : lo - 1];
    O.bwt[U.toff + r + 1] = t[hi == 0 ? U.len - 1 : hi - 1];
  }
  if (lo == 0) O.rank0[gr.unit] = r;
  if (hi == 0) O.rank0[gr.unit] = r + 1;
}

// Run-end pairs (a unlinked: the pair that ends its run) compare their rotations directly, up
// to kPairScan characters, and publish the result for both members (ordat: 1 = this
// rotation first, 2 = the partner first, 0 = undecided) for the rest of the run.
__global__ void __launch_bounds__(kT) k_pair_end(const Grp* __restrict__ L, uint32_t n, SortBufs B,
                                                 const uint32_t* __restrict__ E, uint32_t h0, uint32_t* __restrict__ ordat,
                                                 Grp* __restrict__ lng, uint32_t* __restrict__ nlong) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  Grp gr{0, 0, 0, 0};
  if (g < n) gr = L[g];
  const bool pair = g < n && gr.size == 2;
  Unit U{0, 1, 0, 1};
  uint32_t a = 0, b = 0;
  if (pair) {
    U = B.units[gr.unit];
    a = B.sa[gr.start];
    b = B.sa[gr.start + 1];
  }
  const bool end = pair && E[U.sbase + a] == a;
  const uint8_t* t = B.text + U.toff;
  const int ord = end ? pair_order(t, U.len, a, b, h0, kPairShort) : 0;
  if (end) {
    ordat[U.sbase + a] = ord == 0 ? 0u : ord < 0 ? 1u : 2u;
    ordat[U.sbase + b] = ord == 0 ? 0u : ord < 0 ? 2u : 1u;
  }
  const uint32_t p = wave_append(nlong, end && ord == 0);  // longer comparisons: k_pair_long
  if (end && ord == 0) lng[p] = gr;
}

// Run-end pairs still tied after kPairShort characters (the run ends inside a larger group),
// one wave each: the lanes compare consecutive 16-character pieces, 1024 characters per step.
__global__ void __launch_bounds__(kT) k_pair_long(const Grp* __restrict__ lng, const uint32_t* __restrict__ nlong,
                                                  SortBufs B, uint32_t h0, uint32_t* __restrict__ ordat) {
  const uint32_t wv = blockIdx.x * (kT / 64) + (threadIdx.x >> 6), lane = __lane_id();
  if (wv >= *nlong) return;
  const Grp gr = lng[wv];
  const Unit U = B.units[gr.unit];
  const uint8_t* t = B.text + U.toff;
  const uint32_t a = B.sa[gr.start], b = B.sa[gr.start + 1];
  const uint32_t base = h0 + kPairShort;
  int ord = 0;
  for (uint32_t k = 0; k < kPairScan && ord == 0; k += 64 * 16) {
    const uint32_t off = base + k + 16 * lane;
    uint32_t xe[4], xf[4];
    text_key16(t, U.len, cyc_pos(a, off % U.len, U.len), xe);
    text_key16(t, U.len, cyc_pos(b, off % U.len, U.len), xf);
    int o = 0;
#pragma unroll
    for (int w = 3; w >= 0; w--)
      if (xe[w] != xf[w]) o = xe[w] < xf[w] ? -1 : 1;
    const uint64_t m = __ballot(o != 0);
    if (m) ord = __shfl(o, __ffsll((unsigned long long)m) - 1, 64);
  }
  if (lane == 0) {
    ordat[U.sbase + a] = ord == 0 ? 0u : ord < 0 ? 1u : 2u;
    ordat[U.sbase + b] = ord == 0 ? 0u : ord < 0 ? 2u : 1u;
  }
}

// Every pair takes the order of its run's end pair (a, b) ~ (a + j, b + j): the pairs
// between are tied, so their first characters agree.  Other groups, and pairs left
// undecided, go to R for the doubling.
__global__ void __launch_bounds__(kT) k_pair_resolve(const Grp* __restrict__ L, uint32_t n, SortBufs B, SortOut O,
                                                     const uint32_t* __restrict__ E, const uint32_t* __restrict__ F,
                                                     const uint32_t* __restrict__ ulist_of,
                                                     const uint32_t* __restrict__ tbase,
                                                     const uint32_t* __restrict__ ordat, Grp* __restrict__ R,
                                                     uint32_t* __restrict__ nR) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  Grp gr{0, 0, 0, 0};
  if (g < n) gr = L[g];
  bool keep = g < n && gr.size != 2;
  if (g < n && gr.size == 2) {
    const Unit U = B.units[gr.unit];
    const uint32_t a = B.sa[gr.start], b = B.sa[gr.start + 1];
    uint32_t e = E[U.sbase + a];
    if (e == 0xffffffffu) e = F[tbase[ulist_of[gr.unit]] + a / kRunTile + 1];
    const uint32_t o = ordat[U.sbase + e];
    if (o == 0) {
      keep = true;
    } else {
      const bool a_first = o == 1;
      pair_write(B, O, gr, U, B.text + U.toff, a_first ? a : b, a_first ? b : a);
    }
  }
  const uint32_t p = wave_append(nR, keep);
  if (keep) R[p] = gr;
}

// BWT bytes of the slots of the deep groups (everything else was written when its rotation
// was ordered), for aperiodic units.
__global__ void __launch_bounds__(kT) k_deep_out(const Grp* __restrict__ L0, uint32_t n, const Unit* __restrict__ units,
                                                 const uint32_t* __restrict__ sa, const uint8_t* __restrict__ text,
                                                 uint8_t* __restrict__ bwt) {
  for_members(L0, n, [&](const Grp& g, uint32_t e) {
    const Unit U = units[g.unit];
    if (U.k != 1) return;  // periodic roots: the whole last column is written afterwards
    const uint32_t v = sa[g.start + e];
    bwt[U.toff + g.start + e - U.sbase] = text[U.toff + (v == 0 ? U.len - 1 : v - 1)];
  });
}

// Last column of the listed units from the SA (periodic roots repeated k times).
__global__ void __launch_bounds__(kT) k_unit_out(const uint32_t* __restrict__ ulist, const Unit* __restrict__ units,
                                                 const uint32_t* __restrict__ sa, const uint8_t* __restrict__ text,
                                                 uint8_t* __restrict__ bwt) {
  const Unit U = units[ulist[blockIdx.y]];
  const uint32_t x = blockIdx.x * kT + threadIdx.x;
  if (x >= U.len * U.k) return;
  const uint32_t v = sa[U.sbase + (U.k == 1 ? x : x / U.k)];
  bwt[U.toff + x] = text[U.toff + (v == 0 ? U.len - 1 : v - 1)];
}

// BZG_CHECK diagnostics: every member of group g must equal member 0 on min(depth, 64)
// characters.  res[0] counts violating groups, res[1..4] the first one (start, size, unit, flags).
__global__ void k_check_groups(const Grp* __restrict__ L, uint32_t n, SortBufs B, uint32_t* __restrict__ res) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const Grp gr = L[g];
  if (gr.size < 2) return;
  const Unit U = B.units[gr.unit];
  const uint32_t* src = (gr.flags & kGrpAlt) ? B.sa2 : B.sa;
  auto rot = [&](uint32_t e) { return (gr.flags & kGrpIdent) ? e : src[gr.start + e]; };
  const uint32_t d = min(grp_depth(gr), 64u);
  const uint8_t* t = B.text + U.toff;
  const uint32_t v0 = rot(0);
  bool bad = false;
  for (uint32_t e = 1; e < min(gr.size, 64u) && !bad; e++) {
    const uint32_t v = rot(e);
    if (v >= U.len) { bad = true; break; }
    for (uint32_t c = 0; c < d; c++)
      if (t[(v0 + c) % U.len] != t[(v + c) % U.len]) { bad = true; break; }
  }
  if (bad && atomicAdd(&res[0], 1u) == 0) {
    res[1] = gr.start; res[2] = gr.size; res[3] = gr.unit; res[4] = gr.flags;
  }
}

__global__ void k_rank0_isa(const uint32_t* __restrict__ ulist, uint32_t n, const Unit* __restrict__ units,
                            const uint32_t* __restrict__ isa, uint32_t* __restrict__ rank0) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t u = ulist[i];
  rank0[u] = isa[units[u].sbase] - units[u].sbase;
}

}  // namespace

// ---- quasi-periodic blocks (qsa.h): the analytic order of qsa_plan, written out.  The block's
// unit is a single rotation for the sort (k_init_units finishes it at once); this kernel then
// writes the block's last column and origPtr.  Table of block q at tab + Q.tab: cum (p + 1),
// ord (p), lo (nspec), srot (nspec).
struct QBlock {
  uint32_t toff, n, p, desc, nspec, tab, unit, pad;
};
__global__ void __launch_bounds__(kT) k_qsa(const QBlock* __restrict__ qb, const uint32_t* __restrict__ tab,
                                            const uint8_t* __restrict__ text, uint8_t* __restrict__ bwt,
                                            uint32_t* __restrict__ rank0) {
  const QBlock Q = qb[blockIdx.y];
  const uint32_t* cum = tab + Q.tab;
  const uint32_t* ord = cum + Q.p + 1;
  const uint32_t* lo = ord + Q.p;
  const uint32_t* srot = lo + Q.nspec;
  const uint8_t* t = text + Q.toff;
  const uint32_t nn = Q.n - Q.p + 1;  // normal rotations 0 .. n - p
  for (uint32_t y = blockIdx.x * kT + threadIdx.x; y < nn + Q.nspec; y += gridDim.x * kT) {
    uint32_t rot, fin;
    if (y < nn) {
      const uint32_t k = upper_idx(cum, Q.p, y);
      const uint32_t o = y - cum[k], cnt = cum[k + 1] - cum[k];
      rot = ord[k] + (Q.desc ? cnt - 1 - o : o) * Q.p;
      uint32_t a = 0, b = Q.nspec;  // specials placed before normal y: lo[j] <= y
      while (a < b) {
        const uint32_t m = (a + b) >> 1;
        if (lo[m] <= y) a = m + 1;
        else b = m;
      }
      fin = y + a;
    } else {
      const uint32_t j = y - nn;
      rot = srot[j];
      fin = lo[j] + j;
    }
    bwt[Q.toff + fin] = t[rot == 0 ? Q.n - 1 : rot - 1];
    if (rot == 0) rank0[Q.unit] = fin;
  }
}

// ------------------------------------------------------------------------------------
void bwt_stage(Workspace& ws, const Rle1Result& r, const std::vector<uint32_t>& h_boff,
               const std::vector<uint32_t>& h_period, uint8_t* bwt, uint32_t* rank0, SortStats* stats,
               hipStream_t st, const uint32_t* h_qper) {
  const uint32_t nb = r.nblocks;
  if (nb == 0) return;
  if (nb > 0xffffu) throw HipFailure(hipErrorInvalidValue);  // S2 keys carry 16-bit unit ids
  std::vector<Unit> hu(nb);
  uint64_t S = 0;
  uint32_t maxlen = 0;
  std::vector<uint32_t> periodic, quasi;
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t n_b = h_boff[b + 1] - h_boff[b];
    maxlen = std::max(maxlen, n_b);
    if (h_qper && h_qper[b]) {  // ordered analytically (k_qsa): one slot for the sort
      hu[b] = Unit{(uint32_t)S, 1u, h_boff[b], 1u};
      quasi.push_back(b);
      S += 1;
      continue;
    }
    hu[b] = Unit{(uint32_t)S, h_period[b], h_boff[b], n_b / h_period[b]};
    if (hu[b].k > 1) periodic.push_back(b);
    S += h_period[b];
  }
  Unit* units = ws.typed<Unit>("sort_units", nb);
  HIP_OK(hipMemcpyAsync(units, hu.data(), sizeof(Unit) * nb, hipMemcpyHostToDevice, st));
  // plans of the quasi-periodic blocks from their first period (host, qsa.cpp)
  std::vector<QBlock> hq;
  std::vector<uint32_t> hqt;
  QBlock* dq = nullptr;
  uint32_t* dqt = nullptr;
  uint32_t qmax = 0;
  if (!quasi.empty()) {
    std::vector<uint8_t> wbuf(quasi.size() * kQsaMaxPeriod);
    for (size_t j = 0; j < quasi.size(); j++)
      HIP_OK(hipMemcpyAsync(wbuf.data() + j * kQsaMaxPeriod, r.blk + h_boff[quasi[j]], h_qper[quasi[j]],
                            hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    for (size_t j = 0; j < quasi.size(); j++) {
      const uint32_t b = quasi[j], n_b = h_boff[b + 1] - h_boff[b], p = h_qper[b];
      QsaPlan plan;
      qsa_plan(wbuf.data() + j * kQsaMaxPeriod, p, n_b, plan);
      hq.push_back(QBlock{h_boff[b], n_b, p, plan.desc ? 1u : 0u, p - 1, (uint32_t)hqt.size(), b, 0u});
      hqt.insert(hqt.end(), plan.cum.begin(), plan.cum.end());
      hqt.insert(hqt.end(), plan.ord.begin(), plan.ord.end());
      hqt.insert(hqt.end(), plan.lo.begin(), plan.lo.end());
      hqt.insert(hqt.end(), plan.srot.begin(), plan.srot.end());
      qmax = std::max(qmax, n_b);
    }
    dq = ws.typed<QBlock>("sort_qblk", hq.size());
    dqt = ws.u32("sort_qtab", hqt.size() + 16);
    HIP_OK(hipMemcpyAsync(dq, hq.data(), sizeof(QBlock) * hq.size(), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(dqt, hqt.data(), 4 * hqt.size(), hipMemcpyHostToDevice, st));
  }

  SortBufs B{};
  B.sa = ws.u32("sort_sa", S + 16);
  B.sa2 = ws.u32("sort_sa2", S + 16);
  B.sk = ws.u32("sort_sk", S + 16);
  B.sk2 = ws.u32("sort_sk2", S + 16);
  B.text = r.blk;
  B.units = units;
  // S2 -> S3 handoff depth (profiles/r02_dwave_sweep.txt; 64 / 128 measured slower in round 4;
  // BZG_DWAVE / BZG_DWAVE_TINY: A/B knobs)
  static const uint32_t dwave = (uint32_t)std::max(32ll, env_ll("BZG_DWAVE", 256));
  static const uint32_t dwave_tiny = (uint32_t)std::max(32ll, env_ll("BZG_DWAVE_TINY", 256));
  B.dwave = dwave;
  B.dwave_tiny = dwave_tiny;
  // class lists: a class-c bucket holds more than kClsMax[c-1] rotations
  ClsLists C{};
  size_t ccap[kNCls];
  for (int c = 0; c < kNCls; c++) {
    const uint64_t minsz = c == 0 ? 2 : (uint64_t)kClsMax[c - 1] + 1;
    ccap[c] = S / minsz + nb + 16;
    C.l[c] = ws.typed<Grp>("sort_cls" + std::to_string(c), ccap[c]);
  }
  Grp* nxt6 = ws.typed<Grp>("sort_nxt6", ccap[kClsPacked]);  // (6 / 7 in names: packed / tiled)
  Grp* nxt7 = ws.typed<Grp>("sort_nxt7", ccap[kClsTiled]);
  SortOut O{};
  O.bwt = bwt;
  O.rank0 = rank0;
  O.deep = ws.typed<Grp>("sort_deep", S / 2 + nb + 16);
  O.tdeep = ws.typed<Grp>("sort_tdeep", ccap[0]);
  O.dbg = nullptr;
  if (getenv("BZG_DEBUG")) {
    O.dbg = reinterpret_cast<unsigned long long*>(ws.u32("sort_dbg", 256));
    HIP_OK(hipMemsetAsync(O.dbg, 0, 1024, st));
  }
  // counters: 0..8 class counts (init), 16 class-major scan total, 17 tiles, 18 packed total,
  // 19 n_deep, 20 min depth, 21 / 22 deep pairs, 32 / 33 pair splits (hc 24..30: the S2 class
  // sizes read back)
  uint32_t* cnt = ws.u32("sort_cnt", 64);  // counters: see below; 24..29 S2 class sizes
  O.n_deep = cnt + 19;
  const size_t max_tiles = S / kDTile + ccap[kClsTiled] + 16;
  const size_t max_ptiles = S / kSG + 64;
  const size_t max_tot = ccap[kClsTiled] + max_ptiles;
  uint32_t* TP = ws.u32("sort_TP", max_tiles + 16);
  TileRec* TR = ws.typed<TileRec>("sort_TR", max_tiles + 16);
  uint32_t* hist = ws.u32("sort_hist", max_tiles * 256);
  uint32_t* tot = ws.u32("sort_tot", ccap[kClsTiled] * 256);
  uint32_t* ccnt = ws.u32("sort_ccnt", kNCls * max_tot + 16);
  uint32_t* P = ws.u32("sort_P", ccap[kClsPacked] + 16);
  Unit* gunits = ws.typed<Unit>("sort_gunits", ccap[kClsPacked] + 16);  // the packed groups' units
  uint32_t* first = ws.u32("sort_first", max_ptiles);
  uint32_t* last = ws.u32("sort_last", max_ptiles);
  uint32_t* nrec = ws.u32("sort_nrec", max_ptiles);
  uint32_t* srec = ws.u32("sort_rec", S + 64);  // bucket records of the packed passes and of S2
  uint32_t* scratch =
      ws.u32z("sort_scan", scan_scratch_words(std::max<size_t>(std::max<size_t>(kNCls * max_tot, max_tiles), ccap[kClsPacked])) + 64);
  uint32_t hc[64];
  auto read_counters = [&]() { ws.read_small(hc, cnt, sizeof(hc), st); };
  auto grid = [](uint64_t n) { return (unsigned)std::max<uint64_t>(1, ceil_div64(n, kT)); };
  static const bool debug = getenv("BZG_DEBUG") != nullptr;
  static const bool check = getenv("BZG_CHECK") != nullptr;
  uint32_t* chk = check ? ws.u32("sort_chk", 8) : nullptr;
  auto check_list = [&](const Grp* L, uint32_t n, const char* what, int it, int cls) {
    if (!check || n == 0) return;
    HIP_OK(hipMemsetAsync(chk, 0, 32, st));
    k_check_groups<<<grid(n), kT, 0, st>>>(L, n, B, chk);
    uint32_t h[5];
    HIP_OK(hipMemcpyAsync(h, chk, 20, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (h[0])
      fprintf(stderr, "[bzg check] %s iter %d class %d: %u bad groups of %u; first start %u size %u unit %u depth %u flags %u\n",
              what, it, cls, h[0], n, h[1], h[2], h[3], h[4] >> kGrpDepthShift, h[4] & 31u);
  };

  HIP_OK(hipMemsetAsync(cnt, 0, 64 * 4, st));
  k_init_units<<<grid(nb), kT, 0, st>>>(units, nb, B, O, C, cnt);
  HIP_OK(hipGetLastError());
  read_counters();
  uint32_t ncls[kNCls];
  for (int c = 0; c < kNCls; c++) ncls[c] = hc[c];
  uint32_t n6 = ncls[kClsPacked], n7 = ncls[kClsTiled];
  Grp* cur6 = C.l[kClsPacked];
  Grp* cur7 = C.l[kClsTiled];
  int passes = 0;
  uint64_t s1_elems = 0;
  // ---- S1: byte passes over the buckets larger than kBig (tiled groups > kSG, packed ones <= kSG)
  while (n6 + n7 > 0) {
    ++passes;
    check_list(cur6, n6, "S1 packed", passes, 6);
    check_list(cur7, n7, "S1 tiled", passes, 7);
    k_group_prep<<<grid((uint64_t)n7 + n6), kT, 0, st>>>(cur7, n7, TP, cur6, n6, units, P, gunits);
    HIP_OK(hipGetLastError());
    if (n7) {
      scan_u32(ScanOp::Sum, true, TP, TP, n7, cnt + 17, scratch, st);
      k_tile_owner<<<n7, 64, 0, st>>>(cur7, n7, TP, units, TR);
      HIP_OK(hipGetLastError());
    }
    if (n6) scan_u32(ScanOp::Sum, true, P, P, n6, cnt + 18, scratch, st);
    ws.read_small(hc + 17, cnt + 17, 8, st);
    const uint32_t ntl = n7 ? hc[17] : 0;
    const uint32_t nT = n6 ? ceil_div(hc[18], kSG) : 0;
    // class-major scan over the tiled groups and the packed tiles (tile t at index n7 + t)
    const uint32_t nTot = n7 + nT;
    if (debug) {
      fprintf(stderr, "[bzg sort S1] pass %d: tiled groups=%u tiles=%u | packed groups=%u elems=%u tiles=%u\n", passes,
              n7, ntl, n6, n6 ? hc[18] : 0, nT);
      s1_elems += n6 ? hc[18] : 0;
    }
    if (nT) {
      k_tile_first<<<grid(n6), kT, 0, st>>>(P, n6, cnt + 18, first, last);
      HIP_OK(hipGetLastError());
      k_s1s_pass<<<nT, kTS, 0, st>>>(cur6, gunits, first, last, P, B, O, srec, nrec, ccnt, nTot, n7);
      HIP_OK(hipGetLastError());
    }
    if (n7) {
      k_s1_hist<<<ntl, kT, 0, st>>>(TR, B, hist);
      HIP_OK(hipGetLastError());
      k_s1_off<<<n7, kT, 0, st>>>(cur7, nTot, TP, hist, tot, ccnt, O.deep, O.n_deep);
      HIP_OK(hipGetLastError());
    }
    scan_u32(ScanOp::Sum, true, ccnt, ccnt, (size_t)kNCls * nTot, cnt + 16, scratch, st);
    ClsLists Cp = C;
    for (int c = 0; c < kS2Cls; c++) Cp.base[c] = ncls[c];
    Cp.l[kClsPacked] = nxt6;
    Cp.l[kClsTiled] = nxt7;
    Cp.base[kClsPacked] = Cp.base[kClsTiled] = 0;
    if (n7) {
      k_s1_scatter<<<ntl, kT, 0, st>>>(TR, B, O, hist, tot, ccnt, nTot, Cp);
      HIP_OK(hipGetLastError());
    }
    k_s1_tail<<<n7 + ceil_div(nT, kT / 64), kT, 0, st>>>(cur7, n7, B, tot, S1sEmitArgs{cur6, first, last, P, nT, srec, nrec, n7},
                                                         O, ccnt, nTot, Cp);
    HIP_OK(hipGetLastError());
    // the class bounds of the class-major scan: its entries at c * nTot (class starts) and its total
    uint32_t bnd[kNCls + 1];
    ws.read_small({{bnd, ccnt, 4ull * kNCls, nTot}, {bnd + kNCls, cnt + 16, 4}}, st);
    for (int c = 0; c < kS2Cls; c++) ncls[c] += bnd[c + 1] - bnd[c];
    n6 = bnd[kClsPacked + 1] - bnd[kClsPacked];
    n7 = bnd[kClsTiled + 1] - bnd[kClsTiled];
    std::swap(cur6, nxt6);
    std::swap(cur7, nxt7);
  }
  // ---- S2: every size class
  if (debug)
    fprintf(stderr, "[bzg sort S2] buckets by class: 2-8:%u 9-16:%u 17-32:%u 33-64:%u 65-128:%u 129-256:%u 257-512:%u\n",
            ncls[0], ncls[1], ncls[2], ncls[3], ncls[4], ncls[5], ncls[6]);
  // bitonic rounds before the rank-counting tail (classes 1, 2) or before the still-tied runs
  // are emitted as new groups (classes 3..6, one group per wave; the S2 loop repeats until
  // every list is empty)
  constexpr int kR3 = 8, kR4 = 2, kR5 = 2, kR6 = 2;  // (profiles/r03_*, r04_*: 3 or 4 rounds for class 3 slower)
  {
    ClsLists N{};
    for (int c = 0; c < kS2Cls; c++) N.l[c] = ws.typed<Grp>("sort_s2n" + std::to_string(c), ccap[c]);
    {  // block order for the first S2 round (see k_unit_count)
      // A list of more than S / 32 groups (high-entropy input: millions of small
      // buckets, most of them settled by their first 16 characters) stays as it is: its
      // reorder would cost more than the L2 locality it buys.
      constexpr uint64_t reorder_div = 32;  // profiles/r04_ab_s2_reorder.txt
      // A part of few blocks is skipped as well: its text and slots are few enough to stay in
      // the caches in any order, and the reorder's 7 x 4 launches and its per-block atomics
      // (few counters, heavily contended) cost a 50 MB part about 0.5 ms on its critical path.
      static const uint64_t reorder_min_s = (uint64_t)env_ll("BZG_REORDER_MIN_S", 200000000ll);
      uint32_t* ucnt = ws.u32("sort_ucnt", nb + 64);
      for (int c = 0; c < kS2Cls; c++) {
        if (S < reorder_min_s) break;
        if (ncls[c] < 2) continue;
        if ((uint64_t)ncls[c] * reorder_div > S) continue;
        HIP_OK(hipMemsetAsync(ucnt, 0, 4 * (size_t)nb, st));
        k_unit_count<<<grid(ncls[c]), kT, 0, st>>>(C.l[c], ncls[c], ucnt);
        HIP_OK(hipGetLastError());
        scan_u32(ScanOp::Sum, true, ucnt, ucnt, nb, nullptr, scratch, st);
        k_unit_scatter<<<grid(ncls[c]), kT, 0, st>>>(C.l[c], ncls[c], ucnt, N.l[c]);
        HIP_OK(hipGetLastError());
        std::swap(C.l[c], N.l[c]);
      }
    }
    const size_t max_s2 = ccap[3] + ccap[4] + ccap[5] + ccap[6];
    Grp* tiny2 = ws.typed<Grp>("sort_tiny2", ccap[0]);
    Grp* tiny8 = ws.typed<Grp>("sort_tiny8", ccap[0]);
    uint32_t* ccnt2 = ws.u32("sort_s2cnt", kS2Cls * max_s2 + 16);
    uint32_t* scratch2 = ws.u32z("sort_s2scan", scan_scratch_words(kS2Cls * max_s2 + 16) + 64);
    int s2_iters = 0;
    for (;;) {
      ++s2_iters;
      if (debug)
        fprintf(stderr, "[bzg sort S2] iter %d: 2-8:%u 9-16:%u 17-32:%u 33-64:%u 65-128:%u 129-256:%u 257-512:%u\n",
                s2_iters, ncls[0], ncls[1], ncls[2], ncls[3], ncls[4], ncls[5], ncls[6]);
      for (int c = 0; c < kS2Cls; c++) check_list(C.l[c], ncls[c], "S2", s2_iters, c);
      // the small classes' deep groups, appended by one k_deep_compact_all after all of them
      DeepSrcs D{};
      uint32_t dwg = 0;
      auto add_deep = [&](const Grp* slot, const Grp* in, const uint32_t* num, uint32_t n, uint32_t m) {
        D.s[D.ns++] = DeepSrc{slot, in, num, n, m, dwg};
        dwg += ceil_div(n, kT * kCompactPer);
      };
      if (ncls[0]) {
        // (cnt + 32, + 33: zero at the start and after every iteration's k_s2_emit)
        k_split_pairs<<<ceil_div(ncls[0], kT * kSplitPer), kT, 0, st>>>(C.l[0], ncls[0], tiny2, tiny8, cnt + 32);
        HIP_OK(hipGetLastError());
        uint32_t hn[2];
        ws.read_small(hn, cnt + 32, 8, st);
        if (hn[0]) {
          k_tiny<2><<<ceil_div(hn[0], 32 * (kT / 64)), kT, 0, st>>>(tiny2, hn[0], B, O);
          add_deep(nullptr, O.tdeep, nullptr, hn[0], 0);
        }
        if (hn[1]) {
          SortOut O8 = O;
          O8.dm = 4;
          O8.dslot = ws.typed<Grp>("sort_dslot8", (size_t)hn[1] * 4);
          O8.dnum = ws.u32("sort_dnum8", hn[1]);
          k_tiny<8><<<ceil_div(hn[1], 8 * (kT / 64)), kT, 0, st>>>(tiny8, hn[1], B, O8);
          add_deep(O8.dslot, nullptr, O8.dnum, hn[1], 4u);
        }
      }
      if (ncls[1]) {
        SortOut O1 = O;
        O1.dm = 8;  // a segment of 16 has at most 8 deep groups
        O1.dslot = ws.typed<Grp>("sort_dslot1", (size_t)ncls[1] * O1.dm);
        O1.dnum = ws.u32("sort_dnum1", ncls[1]);
        k_bsort<16, 1, 2, false><<<ceil_div(ncls[1], 4 * (kT / 64)), kT, 0, st>>>(C.l[1], ncls[1], B, O1);
        add_deep(O1.dslot, nullptr, O1.dnum, ncls[1], O1.dm);
      }
      if (ncls[2]) {
        SortOut O2 = O;
        O2.dm = 16;
        O2.dslot = ws.typed<Grp>("sort_dslot2", (size_t)ncls[2] * O2.dm);
        O2.dnum = ws.u32("sort_dnum2", ncls[2]);
        k_bsort<32, 1, 2, false><<<ceil_div(ncls[2], 2 * (kT / 64)), kT, 0, st>>>(C.l[2], ncls[2], B, O2);
        add_deep(O2.dslot, nullptr, O2.dnum, ncls[2], O2.dm);
      }
      if (D.ns) k_deep_compact_all<<<dwg, kT, 0, st>>>(D, O.deep, O.n_deep);
      HIP_OK(hipGetLastError());
      const uint32_t total = ncls[3] + ncls[4] + ncls[5] + ncls[6];
      if (total == 0) break;
      // (every group of the emitting classes writes its kS2Cls counts; the scan's last input
      // word does not affect its exclusive output)
      S2Emit E{srec, ccnt2, total, 0};
      if (ncls[3]) k_bsort<64, 1, kR3, false, true><<<ceil_div(ncls[3], kT / 64), kT, 0, st>>>(C.l[3], ncls[3], B, O, E);
      E.gbase += ncls[3];
      if (ncls[4]) k_bsort<64, 2, kR4, true, true><<<ceil_div(ncls[4], kT / 64), kT, 0, st>>>(C.l[4], ncls[4], B, O, E);
      E.gbase += ncls[4];
      if (ncls[5]) k_bsort<64, 4, kR5, false, true><<<ceil_div(ncls[5], kT / 64), kT, 0, st>>>(C.l[5], ncls[5], B, O, E);
      E.gbase += ncls[5];
      if (ncls[6]) k_bsort<64, 8, kR6, false, true><<<ceil_div(ncls[6], kT / 64), kT, 0, st>>>(C.l[6], ncls[6], B, O, E);
      HIP_OK(hipGetLastError());
      scan_u32(ScanOp::Sum, true, ccnt2, ccnt2, kS2Cls * (size_t)total + 1, nullptr, scratch2, st);
      S2Lists Ls{{C.l[3], C.l[4], C.l[5], C.l[6]},
                 {0, ncls[3], ncls[3] + ncls[4], ncls[3] + ncls[4] + ncls[5], total}};
      k_s2_emit<<<grid(total), kT, 0, st>>>(Ls, srec, ccnt2, total, N, cnt + 32);
      HIP_OK(hipGetLastError());
      // class sizes of the next lists: the class-major scan's entries at c * total
      uint32_t b2[kS2Cls + 1];
      ws.read_small({{b2, ccnt2, 4ull * (kS2Cls + 1), total}}, st);
      for (int c = 0; c < kS2Cls; c++) hc[24 + c] = b2[c + 1] - b2[c];
      for (int c = 0; c < kS2Cls; c++) {
        ncls[c] = hc[24 + c];
        std::swap(C.l[c], N.l[c]);
      }
    }
    if (stats) stats->s2_iters = s2_iters;
    if (debug && O.dbg) {
      unsigned long long d[64];
      HIP_OK(hipMemcpyAsync(d, O.dbg, sizeof(d), hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
      for (int c = 1; c < kS2Cls; c++)
        fprintf(stderr, "[bzg sort S2] class %d waves by round: %llu %llu %llu %llu %llu %llu %llu+ tail %llu\n", c,
                d[8 + 8 * c], d[9 + 8 * c], d[10 + 8 * c], d[11 + 8 * c], d[12 + 8 * c], d[13 + 8 * c], d[14 + 8 * c],
                d[15 + 8 * c]);
      unsigned long long e[64];
      HIP_OK(hipMemcpyAsync(e, O.dbg + 64, sizeof(e), hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
      for (int c = 3; c < kS2Cls; c++) {
        const unsigned long long* x = e + 16 * (c - 3);
        fprintf(stderr, "[bzg sort S2] class %d later rounds: longest run <=4:%llu <=8:%llu <=16:%llu <=32:%llu <=64:%llu >64:%llu"
                " | tied <=4:%llu <=8:%llu <=16:%llu <=32:%llu <=64:%llu >64:%llu\n", c, x[0], x[1], x[2], x[3], x[4], x[5],
                x[8], x[9], x[10], x[11], x[12], x[13]);
      }
    }
  }
  HIP_OK(hipGetLastError());
  read_counters();
  const uint32_t n_deep = hc[19];
  int dbl_iters = 0;
  uint64_t dbl_elems = 0;
  std::vector<uint32_t> fb_units;
  if (n_deep > 0) {
    // ---- S3: prefix doubling for the deep groups, over ISA ranks of the affected units
    B.isa = ws.u32("sort_isa", S + 16);
    B.key = ws.u32("sort_key", S + 16);
    B.key2 = ws.u32("sort_key2", S + 16);
    uint32_t* uflag = ws.u32("sort_uflag", nb + 16);
    HIP_OK(hipMemsetAsync(uflag, 0, 4 * (size_t)nb, st));
    HIP_OK(hipMemsetAsync(cnt + 20, 0xff, 4, st));
    check_list(O.deep, n_deep, "S3 deep", 0, 8);
    k_fb_flag<<<grid(n_deep), kT, 0, st>>>(O.deep, n_deep, uflag, cnt + 20);
    HIP_OK(hipGetLastError());
    std::vector<uint32_t> hf(nb);
    HIP_OK(hipMemcpyAsync(hf.data(), uflag, 4 * (size_t)nb, hipMemcpyDeviceToHost, st));
    read_counters();
    const uint32_t h0 = hc[20];
    uint32_t flen = 0;
    for (uint32_t b = 0; b < nb; b++)
      if (hf[b]) {
        fb_units.push_back(b);
        flen = std::max(flen, hu[b].len * hu[b].k);
      }
    uint32_t* ulist = ws.u32("sort_ulist", fb_units.size() + 16);
    HIP_OK(hipMemcpyAsync(ulist, fb_units.data(), 4 * fb_units.size(), hipMemcpyHostToDevice, st));
    Grp* L0 = ws.typed<Grp>("sort_L0", n_deep + 16);
    if (debug) {  // sizes by source (cache bits of the deep entries: 1 k_tiny, 2 bsort tail, else S1)
      std::vector<Grp> hd(n_deep);
      HIP_OK(hipMemcpyAsync(hd.data(), O.deep, sizeof(Grp) * n_deep, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
      uint64_t h[3][4] = {};
      for (const Grp& g : hd) {
        const uint32_t src = grp_cache(g) == 1 ? 0 : grp_cache(g) == 2 ? 1 : 2;
        h[src][std::min<uint32_t>(g.size, 3)]++;
      }
      for (int k = 0; k < 3; k++)
        fprintf(stderr, "[bzg sort S3] deep from %s: size0 %llu size1 %llu size2 %llu size3+ %llu\n",
                k == 0 ? "tiny" : k == 1 ? "tail" : "s1", (unsigned long long)h[k][0], (unsigned long long)h[k][1],
                (unsigned long long)h[k][2], (unsigned long long)h[k][3]);
    }
    k_fb_copy<<<grid(n_deep), kT, 0, st>>>(O.deep, n_deep, L0, B);
    HIP_OK(hipGetLastError());
    uint32_t n_left = n_deep;
    {  // deep pairs by their run's first mismatch (k_pair_resolve)
      const uint32_t nu = (uint32_t)fb_units.size();
      std::vector<uint32_t> htb(nu + 1, 0u), huo(nb, 0u);
      uint32_t maxt = 0;
      for (uint32_t i = 0; i < nu; i++) {
        const uint32_t nt = ceil_div(hu[fb_units[i]].len, kRunTile);
        htb[i + 1] = htb[i] + nt;
        maxt = std::max(maxt, nt);
        huo[fb_units[i]] = i;
      }
      uint32_t* tbase = ws.u32("sort_p_tbase", nu + 16);
      uint32_t* uof = ws.u32("sort_p_uof", nb + 16);
      uint32_t* tsum = ws.u32("sort_p_tsum", htb[nu] + 16);
      uint32_t* F = ws.u32("sort_p_F", htb[nu] + 16);
      Grp* R = ws.typed<Grp>("sort_p_R", n_deep + 16);
      HIP_OK(hipMemcpyAsync(tbase, htb.data(), 4 * (nu + 1), hipMemcpyHostToDevice, st));
      HIP_OK(hipMemcpyAsync(uof, huo.data(), 4 * nb, hipMemcpyHostToDevice, st));
      uint32_t* pm = B.key;
      uint32_t* E = B.key2;
      const uint32_t pch = ceil_div(flen, kT * 16);
      k_pm_init<<<nu * pch, kT, 0, st>>>(ulist, nu, pch, units, pm);
      k_pair_mark<<<grid(n_deep), kT, 0, st>>>(L0, n_deep, B, pm);
      k_runend_tile<<<dim3(maxt, nu), kT, 0, st>>>(ulist, tbase, nu, units, pm, E, tsum);
      k_runend_tiles<<<dim3(ceil_div(maxt, kT), nu), kT, 0, st>>>(ulist, tbase, nu, units, tsum, F);
      HIP_OK(hipMemsetAsync(cnt + 21, 0, 4, st));
      uint32_t* ordat = B.isa;  // (the ISA is built afterwards, for the groups left)
      HIP_OK(hipMemsetAsync(cnt + 22, 0, 4, st));
      k_pair_end<<<grid(n_deep), kT, 0, st>>>(L0, n_deep, B, E, h0, ordat, R, cnt + 22);
      {  // (R holds the long ones until k_pair_resolve refills it; waves past the count exit)
        uint32_t nlong = 0;
        ws.read_small(&nlong, cnt + 22, 4, st);
        if (nlong) k_pair_long<<<ceil_div(nlong, kT / 64), kT, 0, st>>>(R, cnt + 22, B, h0, ordat);
      }
      k_pair_resolve<<<grid(n_deep), kT, 0, st>>>(L0, n_deep, B, O, E, F, uof, tbase, ordat, R, cnt + 21);
      HIP_OK(hipGetLastError());
      read_counters();
      n_left = hc[21];
      if (debug) fprintf(stderr, "[bzg sort S3] pairs resolved %u of %u deep groups\n", n_deep - n_left, n_deep);
      HIP_OK(hipMemcpyAsync(L0, R, sizeof(Grp) * n_left, hipMemcpyDeviceToDevice, st));
      // the units that still have deep groups
      fb_units.clear();
      flen = 0;
      if (n_left) {
        HIP_OK(hipMemsetAsync(uflag, 0, 4 * (size_t)nb, st));
        HIP_OK(hipMemsetAsync(cnt + 20, 0xff, 4, st));
        k_fb_flag<<<grid(n_left), kT, 0, st>>>(L0, n_left, uflag, cnt + 20);
        HIP_OK(hipGetLastError());
        HIP_OK(hipMemcpyAsync(hf.data(), uflag, 4 * (size_t)nb, hipMemcpyDeviceToHost, st));
        read_counters();  // (L0's flags are reset: h0 stays the minimum depth of the deep list)
        for (uint32_t b = 0; b < nb; b++)
          if (hf[b]) {
            fb_units.push_back(b);
            flen = std::max(flen, hu[b].len * hu[b].k);
          }
        HIP_OK(hipMemcpyAsync(ulist, fb_units.data(), 4 * fb_units.size(), hipMemcpyHostToDevice, st));
      }
    }
    if (n_left > 0) {
    {
      const uint32_t nu = (uint32_t)fb_units.size(), chunks = ceil_div(flen, kT);
      k_fb_isa_all<<<kNumXcd * ceil_div(nu, kNumXcd) * chunks, kT, 0, st>>>(ulist, nu, chunks, units, B);
    }
    HIP_OK(hipGetLastError());
    k_fb_group_isa<<<grid(n_left), kT, 0, st>>>(L0, n_left, B);
    HIP_OK(hipGetLastError());
    if (debug) {
      std::vector<Grp> hd(n_left);
      HIP_OK(hipMemcpyAsync(hd.data(), L0, sizeof(Grp) * n_left, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
      uint64_t tot = 0, mx = 0, hist[5] = {0, 0, 0, 0, 0};
      for (const Grp& g : hd) {
        tot += g.size;
        mx = std::max<uint64_t>(mx, g.size);
        hist[std::min<uint32_t>(g.size, 4)]++;
      }
      fprintf(stderr, "[bzg sort S3] deep groups=%u elems=%llu max=%llu sizes 0:%llu 1:%llu 2:%llu 3:%llu 4+:%llu units=%zu h0=%u\n",
              n_left, (unsigned long long)tot, (unsigned long long)mx, (unsigned long long)hist[0],
              (unsigned long long)hist[1], (unsigned long long)hist[2], (unsigned long long)hist[3],
              (unsigned long long)hist[4], fb_units.size(), h0);
    }
    doubling_sort(ws, B, L0, n_left, h0, &dbl_iters, &dbl_elems, st);
    k_deep_out<<<grid(n_left), kT, 0, st>>>(L0, n_left, units, B.sa, r.blk, bwt);
    HIP_OK(hipGetLastError());
    k_rank0_isa<<<grid(fb_units.size()), kT, 0, st>>>(ulist, (uint32_t)fb_units.size(), units, B.isa, rank0);
    HIP_OK(hipGetLastError());
    }
  }
  if (!quasi.empty()) {
    k_qsa<<<dim3(std::min<uint32_t>(ceil_div(qmax, kT), 1024u), (unsigned)hq.size()), kT, 0, st>>>(dq, dqt, r.blk, bwt,
                                                                                                 rank0);
    HIP_OK(hipGetLastError());  // (the plan tables were copied before the first counter read-back)
  }
  if (!periodic.empty()) {  // periodic roots: the root's last column repeated k times
    uint32_t* plist = ws.u32("sort_plist", periodic.size() + 16);
    HIP_OK(hipMemcpyAsync(plist, periodic.data(), 4 * periodic.size(), hipMemcpyHostToDevice, st));
    k_unit_out<<<dim3(ceil_div(maxlen, kT), (unsigned)periodic.size()), kT, 0, st>>>(plist, units, B.sa, r.blk, bwt);
    HIP_OK(hipGetLastError());
  }
  if (stats) {
    stats->iterations = passes + 1 + dbl_iters;
    stats->unsorted_elems = s1_elems + dbl_elems;
  }
}

}  // namespace bzg
