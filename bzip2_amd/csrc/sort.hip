// sort.hip -- stage A4: batched cyclic suffix sorting (BWT) for all blocks of a batch.
//
// Replaces the reference's divsufsort (blocksort.c:1503-1545).  For an aperiodic block all
// rotations are distinct, so any correct sort yields the reference's last column and
// origPtr (parity fact 3).  Periodic blocks (w^k) are reduced to their
// primitive root w; the tie rank among the k identical copies of rotation 0 is resolved on
// the host (resolver.cpp, A5).
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
//   S3  groups still equal after kDWave characters (long repeats) or S1 buckets still larger
//       than kBig after kDBig characters go to prefix doubling (sortdbl.hip) over ISA ranks
//       built for the affected blocks only.
#include <algorithm>
#include <cstdlib>
#include <string>

#include "scan.h"
#include "sort_common.h"

namespace bzg {

namespace {

constexpr int kT = 256;
constexpr uint32_t kBig = 256;        // buckets larger than this are split by S1 byte passes
constexpr uint32_t kDTile = 4096;     // rotations per workgroup in an S1 pass
constexpr uint32_t kPerT = kDTile / kT;
constexpr uint32_t kDBig = 16;        // S1 byte passes stop at this depth (then doubling)
constexpr uint32_t kDWave = 1024;     // S2 rounds stop at this depth (then doubling)
constexpr int kNCls = 7;              // size classes 0..5 (S2) and 6 (next S1 pass)
constexpr uint32_t kClsMax[6] = {8, 16, 32, 64, 128, 256};

__host__ __device__ __forceinline__ uint32_t size_cls(uint32_t n) {
  return n <= 8 ? 0u : n <= 16 ? 1u : n <= 32 ? 2u : n <= 64 ? 3u : n <= 128 ? 4u : n <= 256 ? 5u : 6u;
}

struct SortOut {
  uint8_t* bwt;      // last column of aperiodic units, same offsets as the blocks
  uint32_t* rank0;   // slot of rotation 0 relative to its unit
  Grp* deep;         // groups left for the doubling fallback
  uint32_t* n_deep;
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

// Big-endian 4 bytes at p (any alignment; every text buffer has >= 16 bytes of padding).
__device__ __forceinline__ uint32_t ld_be4(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  return __builtin_bswap32(__builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3u)));
}

// The 4 characters of the cyclic unit text t[0..len) starting at q (< len).
__device__ __forceinline__ uint32_t text_key4(const uint8_t* t, uint32_t len, uint32_t q) {
  if (q + 4 <= len) return ld_be4(t + q);
  uint32_t k = 0;
  for (uint32_t i = 0; i < 4; i++) k = (k << 8) | t[(q + i) % len];
  return k;
}

// The 16 characters starting at q, as four big-endian words.
__device__ __forceinline__ void text_key16(const uint8_t* t, uint32_t len, uint32_t q, uint32_t (&k)[4]) {
  if (q + 16 <= len) {
    const uintptr_t a = (uintptr_t)(t + q);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
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

__global__ void k_group_tiles(const Grp* __restrict__ L, uint32_t n, uint32_t* __restrict__ cnt) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n) cnt[g] = ceil_div(L[g].size, kDTile);
}

// ---------------------------------------------------------------- S1 byte passes
// Every workgroup takes kDTile rotations of one group; loads are issued kPerT at a time.
__device__ __forceinline__ void s1_load(const SortBufs& B, const Grp& gr, const Unit& U, uint32_t lo, uint32_t hi,
                                        uint32_t (&vv)[kPerT], uint32_t (&dd)[kPerT]) {
  const uint32_t* src = (gr.flags & kGrpAlt) ? B.sa2 : B.sa;
  const bool ident = gr.flags & kGrpIdent;
  const uint32_t depth = grp_depth(gr);
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++) {
    const uint32_t e = lo + i * kT + threadIdx.x;
    vv[i] = e < hi ? (ident ? e : src[gr.start + e]) : 0u;
  }
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++) {
    const uint32_t e = lo + i * kT + threadIdx.x;
    dd[i] = e < hi ? (uint32_t)B.text[U.toff + cyc_pos(vv[i], depth, U.len)] : 0u;
  }
}

__global__ void __launch_bounds__(kT) k_s1_hist(const Grp* __restrict__ G, uint32_t nG, const uint32_t* __restrict__ TP,
                                                SortBufs B, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t g = upper_idx(TP, nG, t);
  const Grp gr = G[g];
  const Unit U = B.units[gr.unit];
  const uint32_t lo = (t - TP[g]) * kDTile, hi = min(gr.size, lo + kDTile);
  h[threadIdx.x] = 0;
  uint32_t vv[kPerT], dd[kPerT];
  s1_load(B, gr, U, lo, hi, vv, dd);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++)
    if (lo + i * kT + threadIdx.x < hi) atomicAdd(&h[dd[i]], 1u);
  __syncthreads();
  hist[(size_t)t * 256 + threadIdx.x] = h[threadIdx.x];
}

__device__ __forceinline__ uint32_t bucket_cls(uint32_t total, uint32_t depth) {
  if (total < 2) return 0xffu;
  const uint32_t c = size_cls(total);
  return (c == 6 && depth >= kDBig) ? 7u : c;  // 7: still big after kDBig characters
}

// One workgroup per group: bucket totals and bases, per-tile offsets, and the number of
// buckets of every size class (class-major: ccnt[c * nG + g]).
__global__ void __launch_bounds__(kT) k_s1_off(const Grp* __restrict__ G, uint32_t nG, const uint32_t* __restrict__ TP,
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
  uint32_t total = 0;
  for (uint32_t t = t0; t < t1; t++) total += hist[(size_t)t * 256 + d];
  const uint32_t incl = block_incl_sum(total, sh, (uint32_t*)nullptr);
  const uint32_t base = gr.start + incl - total;
  tot[(size_t)g * 256 + d] = total;
  uint32_t run = base;
  for (uint32_t t = t0; t < t1; t++) {
    const uint32_t c = hist[(size_t)t * 256 + d];
    hist[(size_t)t * 256 + d] = run;
    run += c;
  }
  const uint32_t depth = grp_depth(gr) + 1;
  const uint32_t cl = bucket_cls(total, depth);
#pragma unroll
  for (int k = 0; k < kNCls; k++) {
    const uint32_t n = (uint32_t)__popcll(__ballot(cl == (uint32_t)k));
    if (__lane_id() == 0 && n) atomicAdd(&cc[k], n);
  }
  if (cl == 7u) {  // rare: a bucket still larger than kBig after kDBig characters
    const uint32_t dst_alt = (gr.flags & kGrpIdent) ? 0u : ((gr.flags & kGrpAlt) ^ 1u);
    deep[atomicAdd(n_deep, 1u)] = Grp{base, total, gr.unit, dst_alt | (depth << 2)};
  }
  __syncthreads();
  if (d < (uint32_t)kNCls) ccnt[(size_t)d * nG + g] = cc[d];
}

// Scatter of one tile into the bucket order; the first tile of a group also emits the
// group's buckets into the class lists (cscan: exclusive scan of ccnt).
__global__ void __launch_bounds__(kT) k_s1_scatter(const Grp* __restrict__ G, uint32_t nG, const uint32_t* __restrict__ TP,
                                                   SortBufs B, SortOut O, const uint32_t* __restrict__ off,
                                                   const uint32_t* __restrict__ tot, const uint32_t* __restrict__ cscan,
                                                   ClsLists C) {
  __shared__ uint32_t cnt[256];
  __shared__ uint32_t base[256];
  __shared__ uint32_t single[256];
  __shared__ uint32_t wc[kT / 64][kNCls + 1];
  const uint32_t t = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t g = upper_idx(TP, nG, t);
  const Grp gr = G[g];
  const Unit U = B.units[gr.unit];
  const uint32_t lo = (t - TP[g]) * kDTile, hi = min(gr.size, lo + kDTile);
  const bool dst_alt = !(gr.flags & kGrpIdent) && !(gr.flags & kGrpAlt);
  uint32_t* dst = dst_alt ? B.sa2 : B.sa;
  const uint32_t d = threadIdx.x;
  const uint32_t total = tot[(size_t)g * 256 + d];
  cnt[d] = 0;
  base[d] = off[(size_t)t * 256 + d];
  single[d] = total == 1;
  uint32_t vv[kPerT], dd[kPerT];
  s1_load(B, gr, U, lo, hi, vv, dd);
  __syncthreads();
  uint32_t pos[kPerT];
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++)
    pos[i] = (lo + i * kT + threadIdx.x < hi) ? base[dd[i]] + atomicAdd(&cnt[dd[i]], 1u) : 0u;
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++) {
    if (lo + i * kT + threadIdx.x < hi) {
      dst[pos[i]] = vv[i];
      // a bucket of one: this rotation is ordered (its primary-SA copy is made by
      // k_s1_single, since other workgroups may still read the primary SA in this pass)
      if (single[dd[i]]) emit_final(B, O, U, gr.unit, pos[i], vv[i], !dst_alt);
    }
  }
  if (t != TP[g]) return;
  // ---- bucket emission (digit order within the group)
  const uint32_t depth = grp_depth(gr) + 1;
  const uint32_t cl = bucket_cls(total, depth);
  const uint32_t w = d >> 6;
  uint32_t rank = 0;
#pragma unroll
  for (int k = 0; k < kNCls; k++) {
    const uint64_t m = __ballot(cl == (uint32_t)k);
    if (cl == (uint32_t)k) rank = (uint32_t)__popcll(m & lanemask_lt());
    if (__lane_id() == 0) wc[w][k] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  if (cl < (uint32_t)kNCls) {
    for (uint32_t x = 0; x < w; x++) rank += wc[x][cl];
    const uint32_t p = C.base[cl] + cscan[(size_t)cl * nG + g] - cscan[(size_t)cl * nG] + rank;
    C.l[cl][p] = Grp{base[d], total, gr.unit, (dst_alt ? kGrpAlt : 0u) | (depth << 2)};
  }
}

__global__ void __launch_bounds__(kT) k_s1_single(const Grp* __restrict__ G, SortBufs B, const uint32_t* __restrict__ tot) {
  __shared__ uint32_t sh[kT / 64];
  const Grp gr = G[blockIdx.x];
  if ((gr.flags & kGrpIdent) || (gr.flags & kGrpAlt)) return;  // pass wrote the primary SA
  const uint32_t total = tot[(size_t)blockIdx.x * 256 + threadIdx.x];
  const uint32_t incl = block_incl_sum(total, sh, (uint32_t*)nullptr);
  const uint32_t s = gr.start + incl - total;
  if (total == 1) B.sa[s] = B.sa2[s];
}

// out[c] = start of class c in the class-major scan (c < kNCls), out[kNCls] = total.
__global__ void k_cls_bounds(const uint32_t* __restrict__ cscan, uint32_t nG, const uint32_t* __restrict__ total,
                             uint32_t* __restrict__ out) {
  const uint32_t c = threadIdx.x;
  if (c < (uint32_t)kNCls) out[c] = cscan[(size_t)c * nG];
  if (c == (uint32_t)kNCls) out[c] = *total;
}

// ---------------------------------------------------------------- S2
__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

// The 8 characters starting at q (< len) as two big-endian words.
__device__ __forceinline__ void text_key8(const uint8_t* t, uint32_t len, uint32_t q, uint32_t& hi, uint32_t& lo) {
  if (q + 8 <= len) {
    const uintptr_t a = (uintptr_t)(t + q);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
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

// ---- tiny buckets: lane l takes rotation l % 8 of bucket 8 * wave + l / 8.  Every step
// compares the next 16 characters with the rotations of its bucket still tied with it
// (same class, named by its first lane) and adds the smaller ones to its position.
__global__ void __launch_bounds__(kT) k_tiny(const Grp* __restrict__ tiny, uint32_t n_tiny, SortBufs B, SortOut O) {
  const uint32_t lane = __lane_id();
  const uint32_t wv = blockIdx.x * (kT / 64) + (threadIdx.x >> 6);
  const uint32_t bi = wv * 8 + lane / 8, el = lane % 8;
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
  Unit U{0, 1, 0, 1};
  if (act) U = B.units[unit];
  const uint8_t* t = B.text + U.toff;
  uint8_t lastc = 0;  // BWT byte of this rotation, loaded with the first key
  if (act) lastc = t[v == 0 ? U.len - 1 : v - 1];
  bool done = !act;
  uint32_t cls = act ? (lane & ~7u) : 0xffffffffu;
  uint32_t pos = 0;
  const int base = (int)(lane & ~7u);
  for (;;) {
    const uint64_t live = __ballot(!done);
    if (live == 0) break;
    if (d >= kDWave) {  // still tied after kDWave characters: leave to the doubling fallback
      if (!done) {
        const uint64_t mates = match_byte(cls, live);
        const uint32_t r = (uint32_t)__popcll(mates & lanemask_lt());
        B.sa[s0 + pos + r] = v;
        if (r == 0) O.deep[atomicAdd(O.n_deep, 1u)] = Grp{s0 + pos, (uint32_t)__popcll(mates), unit, d << 2};
      }
      break;
    }
    uint32_t k[4] = {0u, 0u, 0u, 0u};
    if (!done) text_key16(t, U.len, cyc_pos(v, d, U.len), k);
    const uint64_t khi = ((uint64_t)k[0] << 32) | k[1], klo = ((uint64_t)k[2] << 32) | k[3];
    uint32_t lt = 0, eq = 0, rep = lane;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int src = base + j;
      const uint32_t cj = (uint32_t)__shfl((int)cls, src, 64);
      const uint64_t hj = __shfl(khi, src, 64);
      const uint64_t lj = __shfl(klo, src, 64);
      if (cj == cls) {
        lt += (hj < khi) || (hj == khi && lj < klo);
        if (hj == khi && lj == klo) {
          if (eq == 0) rep = (uint32_t)src;
          eq++;
        }
      }
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

// ---- buckets of 9..256 rotations: one segment of kSeg lanes x kPer registers per bucket
// (64 / kSeg buckets per wave).  Element (lane, r) sits at position p = (lane % kSeg) * kPer
// + r of its segment.  Sort key: (run start, 8 characters, element index); pads sort last.
// Round 1 sorts by the first 8 characters after the bucket's depth; every later round
// re-keys only the runs still tied, 8 characters deeper, and re-sorts (positions of unique
// elements never move since their run start is their own position).
struct BsortKey {
  uint32_t w0;  // run start << 16 | element index (pads: 0xffff << 16)
  uint32_t hi, lo;
};

// (run start, key, index) order; branch-free: (rs:hi) and (lo:idx) as 48-bit integers.
__device__ __forceinline__ bool key_less(const BsortKey& a, const BsortKey& b) {
  const uint64_t a1 = ((uint64_t)(a.w0 >> 16) << 32) | a.hi, b1 = ((uint64_t)(b.w0 >> 16) << 32) | b.hi;
  const uint64_t a2 = ((uint64_t)a.lo << 16) | (a.w0 & 0xffffu), b2 = ((uint64_t)b.lo << 16) | (b.w0 & 0xffffu);
  return (a1 < b1) | ((a1 == b1) & (a2 < b2));
}

// x from lane ^ J (J < 64): DPP within quads, ds_swizzle within 32 lanes, bpermute across.
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t x) {
  if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
  else if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
  else if constexpr (J < 32) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (J << 10) | 0x1F);
  else return (uint32_t)__shfl_xor((int)x, J, 64);
}

template <int kSeg, int kPer, int J>
__device__ __forceinline__ void bitonic_xlane(BsortKey (&K)[kPer], int k, uint32_t sl) {
  constexpr int jl = J / kPer;
  BsortKey o[kPer];
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    o[r].w0 = xor_lane<jl>(K[r].w0);
    o[r].hi = xor_lane<jl>(K[r].hi);
    o[r].lo = xor_lane<jl>(K[r].lo);
  }
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    const uint32_t p = sl * kPer + r;
    const bool keep_min = ((p & J) == 0) == ((p & k) == 0);
    if (keep_min == key_less(o[r], K[r])) K[r] = o[r];
  }
}

template <int kSeg, int kPer, int J>
__device__ __forceinline__ void bitonic_j(BsortKey (&K)[kPer], int k, uint32_t sl) {
  if constexpr (J >= 1) {
    if (J <= (k >> 1)) {
      if constexpr (J < kPer) {  // partner in another register of this lane
#pragma unroll
        for (int r = 0; r < kPer; r++) {
          const int r2 = r ^ J;
          if (r2 > r) {
            const uint32_t p = sl * kPer + r;
            const bool asc = (p & k) == 0;
            const bool sw = asc ? key_less(K[r2], K[r]) : key_less(K[r], K[r2]);
            const BsortKey x = K[r], y = K[r2];
            K[r] = sw ? y : x;
            K[r2] = sw ? x : y;
          }
        }
      } else {
        bitonic_xlane<kSeg, kPer, J>(K, k, sl);
      }
    }
    bitonic_j<kSeg, kPer, J / 2>(K, k, sl);
  }
}

template <int kSeg, int kPer>
__device__ __forceinline__ void bitonic(BsortKey (&K)[kPer]) {
  constexpr int kN = kSeg * kPer;
  const uint32_t sl = __lane_id() % kSeg;
#pragma unroll
  for (int k = 2; k <= kN; k <<= 1) bitonic_j<kSeg, kPer, kN / 2>(K, k, sl);
}

// Runs still tied after kBsRounds bitonic rounds (few rotations, often long repeats) are
// finished in place: every tied rotation ranks itself among the members of its run that are
// still tied with it (same class, named by the lowest position of the class) on the next 16
// characters per step; positions do not move any more, the final slot is run start + rank.
constexpr int kBsRounds = 2;

template <int kSeg, int kPer>
__device__ void bsort_tail(const SortBufs& B, const SortOut& O, const Grp& g, const Unit& U, uint32_t depth,
                           const BsortKey (&K)[kPer], const bool (&done)[kPer], const uint32_t (&rsn)[kPer],
                           const uint32_t* Lv, uint32_t* Lk, uint4* TK, uint32_t* TC) {
  constexpr int kN = kSeg * kPer;
  const uint32_t lane = __lane_id(), sl = lane % kSeg, sb = (lane / kSeg) * kN;
  const uint8_t* t = B.text + U.toff;
  bool live[kPer];
  uint32_t v[kPer], pos[kPer], cls[kPer], rlen[kPer];
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    live[r] = !done[r] && (K[r].w0 >> 16) != 0xffffu;
    v[r] = live[r] ? Lv[K[r].w0 & 0xffffu] : 0u;
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
    const bool deep = depth >= kDWave;
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      const uint32_t wp = sb + sl * kPer + r;
      uint32_t k[4] = {0u, 0u, 0u, 0u};
      if (live[r] && !deep) text_key16(t, U.len, cyc_pos(v[r], depth, U.len), k);
      TK[wp] = make_uint4(k[0], k[1], k[2], k[3]);
      TC[wp] = live[r] ? cls[r] : 0xffffffffu;
    }
    wave_sync();
    if (deep) {  // still tied after kDWave characters: leave to the doubling fallback
#pragma unroll
      for (int r = 0; r < kPer; r++)
        if (live[r]) {
          const uint32_t p = sl * kPer + r;
          uint32_t rank = 0, cnt = 0;
          for (uint32_t q = rsn[r]; q < rsn[r] + rlen[r]; q++)
            if (TC[sb + q] == cls[r]) {
              cnt++;
              rank += q < p;
            }
          B.sa[g.start + pos[r] + rank] = v[r];
          if (rank == 0) O.deep[atomicAdd(O.n_deep, 1u)] = Grp{g.start + pos[r], cnt, g.unit, depth << 2};
        }
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

template <int kSeg, int kPer>
__global__ void __launch_bounds__(kT) k_bsort(const Grp* __restrict__ L, uint32_t nL, SortBufs B, SortOut O) {
  constexpr int kBPW = 64 / kSeg;
  constexpr int kE = 64 * kPer;  // elements per wave
  __shared__ uint32_t Lv[kT / 64][kE];
  __shared__ uint8_t Lc[kT / 64][kE];
  __shared__ uint32_t Lk[kT / 64][kE];
  __shared__ uint4 TK[kT / 64][kE];
  __shared__ uint32_t TC[kT / 64][kE];
  const uint32_t w = threadIdx.x >> 6, lane = __lane_id();
  const uint32_t sl = lane % kSeg;
  const uint32_t bi = (blockIdx.x * (kT / 64) + w) * kBPW + lane / kSeg;
  const bool has = bi < nL;
  if (__ballot(has) == 0) return;
  Grp g{0, 0, 0, 0};
  if (has) g = L[bi];
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
    K[r].w0 = (valid ? 0u : 0xffff0000u) | idx;
    K[r].hi = hi;
    K[r].lo = lo;
  }
  bool done[kPer];
#pragma unroll
  for (int r = 0; r < kPer; r++) done[r] = false;
  int round = 0;
  for (;;) {
    bitonic<kSeg, kPer>(K);
    // ties with the previous / next position of the segment (same run start and key)
    bool tp[kPer], tn[kPer];
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      BsortKey q;
      if (r > 0) {
        q = K[r - 1];
      } else {
        q.w0 = (uint32_t)__shfl_up((int)K[kPer - 1].w0, 1, 64);
        q.hi = (uint32_t)__shfl_up((int)K[kPer - 1].hi, 1, 64);
        q.lo = (uint32_t)__shfl_up((int)K[kPer - 1].lo, 1, 64);
        if (sl == 0) q.w0 = 0xfffe0000u;  // no previous element
      }
      tp[r] = (K[r].w0 >> 16) != 0xffffu && (q.w0 >> 16) == (K[r].w0 >> 16) && q.hi == K[r].hi && q.lo == K[r].lo;
    }
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      if (r + 1 < kPer) {
        tn[r] = tp[r + 1];
      } else {
        bool x = __shfl_down((int)tp[0], 1, 64) != 0;
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
    uint32_t pre = mx;
#pragma unroll
    for (int o = 1; o < kSeg; o <<= 1) {
      const uint32_t x = (uint32_t)__shfl_up((int)pre, o, 64);
      if (sl >= (uint32_t)o) pre = max(pre, x);
    }
    pre = (uint32_t)__shfl_up((int)pre, 1, 64);
    if (sl == 0) pre = 0;
    bool any_tied = false;
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      rsn[r] = max(rsn[r], pre);
      const uint32_t idx = K[r].w0 & 0xffffu;
      const bool valid = (K[r].w0 >> 16) != 0xffffu;
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
    if (__ballot(any_tied) == 0) break;
    depth += 8;  // tied runs are equal to this depth
    if (++round >= kBsRounds || depth >= kDWave) {
      bsort_tail<kSeg, kPer>(B, O, g, U, depth, K, done, rsn, Lv[w], Lk[w], TK[w], TC[w]);
      break;
    }
    // re-key the tied runs 8 characters deeper; unique elements keep their own position as run start
#pragma unroll
    for (int r = 0; r < kPer; r++) {
      const uint32_t idx = K[r].w0 & 0xffffu;
      const bool valid = (K[r].w0 >> 16) != 0xffffu;
      if (!valid) continue;
      const uint32_t p = sl * kPer + r;
      if (done[r]) {
        K[r].w0 = (p << 16) | idx;
        K[r].hi = K[r].lo = 0;
      } else {
        uint32_t hi, lo;
        text_key8(t, U.len, cyc_pos(Lv[w][idx], depth, U.len), hi, lo);
        K[r].w0 = (rsn[r] << 16) | idx;
        K[r].hi = hi;
        K[r].lo = lo;
      }
    }
  }
}

// ---------------------------------------------------------------- fallback glue
__global__ void k_fb_flag(const Grp* __restrict__ D, uint32_t n, uint32_t* __restrict__ uflag, uint32_t* __restrict__ mind) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const Grp gr = D[g];
  uflag[gr.unit] = 1;
  atomicMin(mind, grp_depth(gr));
}

// Deep groups whose data is in the alternate buffer move to the primary SA; the doubling
// list gets the groups with their flags reset.  One workgroup per group.
__global__ void __launch_bounds__(kT) k_fb_copy(const Grp* __restrict__ D, Grp* __restrict__ L0, SortBufs B) {
  const Grp gr = D[blockIdx.x];
  if (gr.flags & kGrpAlt)
    for (uint32_t e = threadIdx.x; e < gr.size; e += kT) B.sa[gr.start + e] = B.sa2[gr.start + e];
  if (threadIdx.x == 0) L0[blockIdx.x] = Grp{gr.start, gr.size, gr.unit, 0};
}

// Members of a deep group take the group's first slot as rank (after k_fb_isa_all).
__global__ void __launch_bounds__(kT) k_fb_group_isa(const Grp* __restrict__ L0, SortBufs B) {
  const Grp gr = L0[blockIdx.x];
  const uint32_t sb = B.units[gr.unit].sbase;
  for (uint32_t e = threadIdx.x; e < gr.size; e += kT) B.isa[sb + B.sa[gr.start + e]] = gr.start;
}

// ISA of every slot of the listed units from the (complete, primary) SA: every rotation's own
// slot; deep groups' members are overwritten afterwards by k_fb_group_isa.
__global__ void __launch_bounds__(kT) k_fb_isa_all(const uint32_t* __restrict__ ulist, const Unit* __restrict__ units,
                                                   SortBufs B) {
  const Unit U = units[ulist[blockIdx.y]];
  const uint32_t q = blockIdx.x * kT + threadIdx.x;
  if (q >= U.len) return;
  const uint32_t v = B.sa[U.sbase + q];
  B.isa[U.sbase + v] = U.sbase + q;
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

__global__ void k_rank0_isa(const uint32_t* __restrict__ ulist, uint32_t n, const Unit* __restrict__ units,
                            const uint32_t* __restrict__ isa, uint32_t* __restrict__ rank0) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t u = ulist[i];
  rank0[u] = isa[units[u].sbase] - units[u].sbase;
}

}  // namespace

// ------------------------------------------------------------------------------------
void bwt_stage(Workspace& ws, const Rle1Result& r, const std::vector<uint32_t>& h_boff,
               const std::vector<uint32_t>& h_period, uint8_t* bwt, uint32_t* rank0, SortStats* stats,
               hipStream_t st) {
  const uint32_t nb = r.nblocks;
  if (nb == 0) return;
  if (nb > 0xffffu) throw HipFailure(hipErrorInvalidValue);  // S2 keys carry 16-bit unit ids
  std::vector<Unit> hu(nb);
  uint64_t S = 0;
  uint32_t maxlen = 0;
  std::vector<uint32_t> periodic;
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t n_b = h_boff[b + 1] - h_boff[b];
    hu[b] = Unit{(uint32_t)S, h_period[b], h_boff[b], n_b / h_period[b]};
    if (hu[b].k > 1) periodic.push_back(b);
    S += h_period[b];
    maxlen = std::max(maxlen, n_b);
  }
  Unit* units = ws.typed<Unit>("sort_units", nb);
  HIP_OK(hipMemcpyAsync(units, hu.data(), sizeof(Unit) * nb, hipMemcpyHostToDevice, st));

  SortBufs B{};
  B.sa = ws.u32("sort_sa", S + 16);
  B.sa2 = ws.u32("sort_sa2", S + 16);
  B.text = r.blk;
  B.units = units;
  // class lists: a class-c bucket holds more than kClsMax[c-1] rotations
  ClsLists C{};
  size_t ccap[kNCls];
  for (int c = 0; c < kNCls; c++) {
    const uint64_t minsz = c == 0 ? 2 : (uint64_t)kClsMax[c - 1] + 1;
    ccap[c] = S / minsz + nb + 16;
    C.l[c] = ws.typed<Grp>("sort_cls" + std::to_string(c), ccap[c]);
  }
  Grp* next = ws.typed<Grp>("sort_next", ccap[6]);
  SortOut O{};
  O.bwt = bwt;
  O.rank0 = rank0;
  O.deep = ws.typed<Grp>("sort_deep", S / 2 + nb + 16);
  uint32_t* cnt = ws.u32("sort_cnt", 64);  // 0..6 class counts (init), 8..15 class bounds, 16 n_deep, 17 tiles, 18 min depth
  O.n_deep = cnt + 16;
  const size_t max_tiles = S / kDTile + ccap[6] + 16;
  uint32_t* TP = ws.u32("sort_TP", max_tiles + 16);
  uint32_t* hist = ws.u32("sort_hist", max_tiles * 256);
  uint32_t* tot = ws.u32("sort_tot", ccap[6] * 256);
  uint32_t* ccnt = ws.u32("sort_ccnt", kNCls * ccap[6] + 16);
  uint32_t* scratch = ws.u32("sort_scan", scan_scratch_words(std::max<size_t>(kNCls * ccap[6], max_tiles)) + 64);
  uint32_t hc[24];
  auto read_counters = [&]() {
    HIP_OK(hipMemcpyAsync(hc, cnt, sizeof(hc), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  };
  auto grid = [](uint64_t n) { return (unsigned)std::max<uint64_t>(1, ceil_div64(n, kT)); };
  static const bool debug = getenv("BZG_DEBUG") != nullptr;

  HIP_OK(hipMemsetAsync(cnt, 0, 64 * 4, st));
  k_init_units<<<grid(nb), kT, 0, st>>>(units, nb, B, O, C, cnt);
  HIP_OK(hipGetLastError());
  read_counters();
  uint32_t ncls[kNCls];
  for (int c = 0; c < kNCls; c++) ncls[c] = hc[c];
  uint32_t n_big = ncls[6];
  Grp* big = C.l[6];
  Grp* nxt = next;
  int passes = 0;
  uint64_t s1_elems = 0;
  // ---- S1: byte passes over the buckets larger than kBig
  while (n_big > 0) {
    ++passes;
    k_group_tiles<<<grid(n_big), kT, 0, st>>>(big, n_big, TP);
    HIP_OK(hipGetLastError());
    scan_u32(ScanOp::Sum, true, TP, TP, n_big, cnt + 17, scratch, st);
    read_counters();
    const uint32_t ntiles = hc[17];
    if (debug) {
      std::vector<Grp> hg(n_big);
      HIP_OK(hipMemcpy(hg.data(), big, sizeof(Grp) * n_big, hipMemcpyDeviceToHost));
      uint64_t el = 0;
      for (const Grp& g : hg) el += g.size;
      s1_elems += el;
      fprintf(stderr, "[bzg sort S1] pass %d: groups=%u elems=%lu tiles=%u\n", passes, n_big, el, ntiles);
    }
    k_s1_hist<<<ntiles, kT, 0, st>>>(big, n_big, TP, B, hist);
    HIP_OK(hipGetLastError());
    k_s1_off<<<n_big, kT, 0, st>>>(big, n_big, TP, hist, tot, ccnt, O.deep, O.n_deep);
    HIP_OK(hipGetLastError());
    scan_u32(ScanOp::Sum, true, ccnt, ccnt, (size_t)kNCls * n_big, cnt + 15, scratch, st);
    k_cls_bounds<<<1, 64, 0, st>>>(ccnt, n_big, cnt + 15, cnt + 8);
    HIP_OK(hipGetLastError());
    ClsLists Cp = C;
    for (int c = 0; c < 6; c++) Cp.base[c] = ncls[c];
    Cp.l[6] = nxt;
    Cp.base[6] = 0;
    k_s1_scatter<<<ntiles, kT, 0, st>>>(big, n_big, TP, B, O, hist, tot, ccnt, Cp);
    HIP_OK(hipGetLastError());
    k_s1_single<<<n_big, kT, 0, st>>>(big, B, tot);
    HIP_OK(hipGetLastError());
    read_counters();
    for (int c = 0; c < 6; c++) ncls[c] += hc[8 + c + 1] - hc[8 + c];
    n_big = hc[8 + kNCls] - hc[8 + 6];
    std::swap(big, nxt);
  }
  // ---- S2: every size class
  if (debug)
    fprintf(stderr, "[bzg sort S2] buckets by class: 2-8:%u 9-16:%u 17-32:%u 33-64:%u 65-128:%u 129-256:%u\n", ncls[0],
            ncls[1], ncls[2], ncls[3], ncls[4], ncls[5]);
  if (ncls[0]) k_tiny<<<ceil_div(ncls[0], 8 * (kT / 64)), kT, 0, st>>>(C.l[0], ncls[0], B, O);
  if (ncls[1]) k_bsort<16, 1><<<ceil_div(ncls[1], 4 * (kT / 64)), kT, 0, st>>>(C.l[1], ncls[1], B, O);
  if (ncls[2]) k_bsort<32, 1><<<ceil_div(ncls[2], 2 * (kT / 64)), kT, 0, st>>>(C.l[2], ncls[2], B, O);
  if (ncls[3]) k_bsort<64, 1><<<ceil_div(ncls[3], kT / 64), kT, 0, st>>>(C.l[3], ncls[3], B, O);
  if (ncls[4]) k_bsort<64, 2><<<ceil_div(ncls[4], kT / 64), kT, 0, st>>>(C.l[4], ncls[4], B, O);
  if (ncls[5]) k_bsort<64, 4><<<ceil_div(ncls[5], kT / 64), kT, 0, st>>>(C.l[5], ncls[5], B, O);
  HIP_OK(hipGetLastError());
  read_counters();
  const uint32_t n_deep = hc[16];
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
    HIP_OK(hipMemsetAsync(cnt + 18, 0xff, 4, st));
    k_fb_flag<<<grid(n_deep), kT, 0, st>>>(O.deep, n_deep, uflag, cnt + 18);
    HIP_OK(hipGetLastError());
    std::vector<uint32_t> hf(nb);
    HIP_OK(hipMemcpyAsync(hf.data(), uflag, 4 * (size_t)nb, hipMemcpyDeviceToHost, st));
    read_counters();
    const uint32_t h0 = hc[18];
    uint32_t flen = 0;
    for (uint32_t b = 0; b < nb; b++)
      if (hf[b]) {
        fb_units.push_back(b);
        flen = std::max(flen, hu[b].len * hu[b].k);
      }
    uint32_t* ulist = ws.u32("sort_ulist", fb_units.size() + 16);
    HIP_OK(hipMemcpyAsync(ulist, fb_units.data(), 4 * fb_units.size(), hipMemcpyHostToDevice, st));
    Grp* L0 = ws.typed<Grp>("sort_L0", n_deep + 16);
    k_fb_copy<<<n_deep, kT, 0, st>>>(O.deep, L0, B);
    HIP_OK(hipGetLastError());
    k_fb_isa_all<<<dim3(ceil_div(flen, kT), (unsigned)fb_units.size()), kT, 0, st>>>(ulist, units, B);
    HIP_OK(hipGetLastError());
    k_fb_group_isa<<<n_deep, kT, 0, st>>>(L0, B);
    HIP_OK(hipGetLastError());
    if (debug) fprintf(stderr, "[bzg sort S3] deep groups=%u units=%zu h0=%u\n", n_deep, fb_units.size(), h0);
    doubling_sort(ws, B, L0, n_deep, h0, &dbl_iters, &dbl_elems, st);
    k_unit_out<<<dim3(ceil_div(flen, kT), (unsigned)fb_units.size()), kT, 0, st>>>(ulist, units, B.sa, r.blk, bwt);
    HIP_OK(hipGetLastError());
    k_rank0_isa<<<grid(fb_units.size()), kT, 0, st>>>(ulist, (uint32_t)fb_units.size(), units, B.isa, rank0);
    HIP_OK(hipGetLastError());
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
