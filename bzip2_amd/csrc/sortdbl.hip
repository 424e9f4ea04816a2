// sortdbl.hip -- A4 fallback: prefix doubling for groups that the text-key string sort
// (sort.hip) leaves unresolved at a large depth (long repeats inside a block).
//
// Manber-Myers / Larsson-Sadakane over the unresolved groups of every affected unit at once:
//   * ISA[sbase_u + i] holds the first slot of i's group ("rank"), consistent with the true
//     order of rotations at depth >= h for every unresolved group;
//   * iteration h: every member of an unsorted group is keyed by rank(i + h); groups larger
//     than kSmall are split by global MSD counting passes on key digits; groups/buckets of
//     <= kSmall elements are packed into LDS tiles and finished by an in-LDS stable LSD radix
//     sort on (item, key);
//   * new groups of size >= 2 form the next iteration's list; h doubles.
// All keys of an iteration are gathered before any rank is rewritten.  The reference's
// divsufsort (blocksort.c:1503-1545) yields the same order: rotations of an aperiodic unit
// are distinct, so any correct sort gives its last column and origPtr.
#include <algorithm>
#include <cstdlib>

#include "scan.h"
#include "sort_common.h"

namespace bzg {

namespace {

constexpr int kT = 256;
constexpr uint32_t kSmall = 1024;   // max group size sorted in LDS
constexpr uint32_t kWin = 1008;     // nominal tile window (tile <= kWin + kSmall - 1 elements)
constexpr uint32_t kTileCap = 2048;
constexpr uint32_t kPer = kTileCap / kT;  // tile elements per thread
constexpr uint32_t kWaveSpan = kTileCap / (kT / 64);  // tile elements per wave in the radix
static_assert(kWin + kSmall - 1 <= kTileCap && kPer % 4 == 0, "tile shape");
constexpr uint32_t kDTile = 4096;   // elements per tile of a digit pass
constexpr uint32_t kRankMax = 48;   // tiles whose groups are all this small sort by rank counting

__global__ void k_group_sizes(const Grp* __restrict__ L, uint32_t n, uint32_t* __restrict__ sizes) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n) sizes[g] = L[g].size;
}

__global__ void k_group_tiles(const Grp* __restrict__ L, uint32_t n, uint32_t* __restrict__ cnt) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n) cnt[g] = ceil_div(L[g].size, kDTile);
}

// Element -> group map: gmap[P[g]] = g on a zeroed array, then an inclusive max-scan.
__global__ void k_mark_groups(const uint32_t* __restrict__ P, uint32_t nL, uint32_t* __restrict__ gmap) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < nL) gmap[P[g]] = g;
}

// key[s] for every member of every group in L.
__global__ void __launch_bounds__(kT) k_gather(const Grp* __restrict__ L, const uint32_t* __restrict__ P,
                                               const uint32_t* __restrict__ gmap, uint32_t total, uint32_t h,
                                               SortBufs B) {
  uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= total) return;
  const uint32_t g = gmap[x];
  const Grp G = L[g];
  const uint32_t s = G.start + (x - P[g]);
  const Unit U = B.units[G.unit];
  const uint32_t i = B.sa[s];
  uint32_t hh = h % U.len;
  uint32_t j = i + hh;
  if (j >= U.len) j -= U.len;
  const uint32_t k = B.isa[U.sbase + j] - U.sbase;
  B.key[s] = k;
}

// Groups too large for an LDS tile go to the digit passes; the rest are tile-sorted in place
// from L (the tiles skip the large ones).  Large groups are rare, so appends are cheap.
__global__ void k_extract_large(const Grp* __restrict__ L, uint32_t nL, int force_all, Grp* __restrict__ large,
                                uint32_t* __restrict__ n_large) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = g < nL;
  Grp G{0, 0, 0, 0};
  if (valid) G = L[g];
  const bool big = valid && (force_all || G.size > kSmall);
  const uint32_t pl = wave_append(n_large, big);
  if (big) large[pl] = G;
}

// ---------------------------------------------------------------- digit passes (large)
__global__ void __launch_bounds__(kT) k_dhist(const Grp* __restrict__ G, uint32_t nG, const uint32_t* __restrict__ TP,
                                              uint32_t shift, SortBufs B, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const uint32_t t = blockIdx.x;
  const uint32_t g = upper_idx(TP, nG, t);
  const Grp gr = G[g];
  const uint32_t c = t - TP[g];
  const uint32_t lo = c * kDTile, hi = min(gr.size, lo + kDTile);
  const uint32_t* kk = (gr.flags & 1) ? B.key2 : B.key;
  h[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t e = lo + threadIdx.x; e < hi; e += kT) atomicAdd(&h[(kk[gr.start + e] >> shift) & 255u], 1u);
  __syncthreads();
  hist[(size_t)t * 256 + threadIdx.x] = h[threadIdx.x];
}

// One workgroup per large group: bucket bases, per-tile offsets, bucket emission.
// mode 0: emit small buckets to `small`, large to `next`;  mode 1 (forced): all to `next`;
// mode 2 (last digit): small to `small`, large to `equal`.
__global__ void __launch_bounds__(kT) k_doff(const Grp* __restrict__ G, uint32_t nG, const uint32_t* __restrict__ TP,
                                             uint32_t* __restrict__ hist, uint32_t* __restrict__ tot, int mode,
                                             Grp* __restrict__ small, uint32_t* __restrict__ n_small,
                                             Grp* __restrict__ next, uint32_t* __restrict__ n_next,
                                             Grp* __restrict__ equal, uint32_t* __restrict__ n_equal) {
  __shared__ uint32_t sh[kT / 64];
  const uint32_t g = blockIdx.x;
  const Grp gr = G[g];
  const uint32_t t0 = TP[g], t1 = t0 + ceil_div(gr.size, kDTile);
  const uint32_t d = threadIdx.x;
  uint32_t total = 0;
  for (uint32_t t = t0; t < t1; t++) total += hist[(size_t)t * 256 + d];
  uint32_t incl = block_incl_sum(total, sh, (uint32_t*)nullptr);
  uint32_t base = gr.start + incl - total;
  tot[(size_t)g * 256 + d] = total;
  uint32_t run = base;
  for (uint32_t t = t0; t < t1; t++) {
    uint32_t c = hist[(size_t)t * 256 + d];
    hist[(size_t)t * 256 + d] = run;
    run += c;
  }
  const Grp nb{base, total, gr.unit, gr.flags ^ 1u};
  const bool emit = total >= 2;
  const bool to_next = emit && (mode == 1 || (total > kSmall && mode == 0));
  const bool to_small = emit && !to_next && total <= kSmall;
  const bool to_equal = emit && !to_next && !to_small;
  const uint32_t pn = wave_append(n_next, to_next);
  const uint32_t ps = wave_append(n_small, to_small);
  const uint32_t pe = wave_append(n_equal, to_equal);
  if (to_next) next[pn] = nb;
  if (to_small) small[ps] = nb;
  if (to_equal) equal[pe] = nb;
}

__global__ void __launch_bounds__(kT) k_dscatter(const Grp* __restrict__ G, uint32_t nG, const uint32_t* __restrict__ TP,
                                                 uint32_t shift, SortBufs B, const uint32_t* __restrict__ off,
                                                 const uint32_t* __restrict__ tot) {
  __shared__ uint32_t cnt[256];
  __shared__ uint32_t base[256];
  __shared__ uint32_t single[256];
  const uint32_t t = blockIdx.x;
  const uint32_t g = upper_idx(TP, nG, t);
  const Grp gr = G[g];
  const uint32_t c = t - TP[g];
  const uint32_t lo = c * kDTile, hi = min(gr.size, lo + kDTile);
  const bool alt = gr.flags & 1;
  const uint32_t* ks = alt ? B.key2 : B.key;
  const uint32_t* vs = alt ? B.sa2 : B.sa;
  uint32_t* kd = alt ? B.key : B.key2;
  uint32_t* vd = alt ? B.sa : B.sa2;
  cnt[threadIdx.x] = 0;
  base[threadIdx.x] = off[(size_t)t * 256 + threadIdx.x];
  single[threadIdx.x] = tot[(size_t)g * 256 + threadIdx.x] == 1;
  __syncthreads();
  const uint32_t sb = B.units[gr.unit].sbase;
  for (uint32_t e = lo + threadIdx.x; e < hi; e += kT) {
    const uint32_t k = ks[gr.start + e], v = vs[gr.start + e];
    const uint32_t d = (k >> shift) & 255u;
    const uint32_t pos = base[d] + atomicAdd(&cnt[d], 1u);
    kd[pos] = k;
    vd[pos] = v;
    if (single[d]) B.isa[sb + v] = pos;  // a bucket of one: its rotation is now fully ordered
  }
}

// Singletons scattered into the alt buffers move to the primary SA.  (Writing them to the
// primary SA inside k_dscatter would race with other workgroups still reading it.)
__global__ void __launch_bounds__(kT) k_dsingle(const Grp* __restrict__ G, uint32_t nG, const uint32_t* __restrict__ TP,
                                                SortBufs B, const uint32_t* __restrict__ tot) {
  __shared__ uint32_t base[257];
  __shared__ uint32_t sh[kT / 64];
  const uint32_t t = blockIdx.x;
  const uint32_t g = upper_idx(TP, nG, t);
  const Grp gr = G[g];
  if (gr.flags & 1) return;  // data came from alt: singletons already landed in the primary SA
  const uint32_t c = t - TP[g];
  const uint32_t lo = c * kDTile, hi = min(gr.size, lo + kDTile);
  const uint32_t tv = tot[(size_t)g * 256 + threadIdx.x];
  const uint32_t incl = block_incl_sum(tv, sh, (uint32_t*)nullptr);
  base[threadIdx.x] = incl - tv;
  if (threadIdx.x == kT - 1) base[256] = incl;
  __syncthreads();
  for (uint32_t e = lo + threadIdx.x; e < hi; e += kT) {
    uint32_t a = 0, b = 256;  // bucket d with base[d] <= e < base[d+1]
    while (b - a > 1) {
      const uint32_t m = (a + b) >> 1;
      if (base[m] <= e) a = m;
      else b = m;
    }
    if (base[a + 1] - base[a] == 1) B.sa[gr.start + e] = B.sa2[gr.start + e];
  }
}

// ---------------------------------------------------------------- small groups (LDS)
// tile index of item i = P[i] / kWin; mark the first item of each tile and one past its last,
// and every tile of the ntiles that no item starts in (inside a large item, or after the last
// one) empty, so that `first` needs no clearing.
__global__ void k_tile_first(const uint32_t* __restrict__ P, uint32_t n, uint32_t ntiles, uint32_t* __restrict__ first,
                             uint32_t* __restrict__ last) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t t = P[i] / kWin;
  if (i == 0 || P[i - 1] / kWin != t) first[t] = i;
  if (i == n - 1 || P[i + 1] / kWin != t) last[t] = i + 1;
  const uint32_t tn = i + 1 < n ? P[i + 1] / kWin : ntiles;
  for (uint32_t e = t + 1; e < tn; e++) first[e] = 0xffffffffu;
}

struct TileLds {
  uint32_t keyA[kTileCap], valA[kTileCap], keyB[kTileCap], valB[kTileCap];
  uint16_t hist[4][256];  // per-wave digit counts / bases (<= kTileCap)
  // items start inside a kWin window and hold >= 2 elements: at most kWin / 2 per tile
  uint32_t ioff[kWin / 2 + 1];  // tile-local offset of each item (+ end)
  uint32_t istart[kWin / 2];
  uint32_t iunit[kWin / 2];
  uint32_t sh[kT / 64];
  uint32_t misc[4];
};

// Stable LSD radix sort of n (<= kTileCap) (key, val) pairs in LDS over bits [0, nbits).
// 4 waves; wave w owns elements [w*kWaveSpan, (w+1)*kWaveSpan), visited 64 at a time in order.
__device__ void lds_radix_sort(TileLds& S, uint32_t n, uint32_t nbits, uint32_t*& keys, uint32_t*& vals) {
  uint32_t* kin = S.keyA;
  uint32_t* vin = S.valA;
  uint32_t* kout = S.keyB;
  uint32_t* vout = S.valB;
  const uint32_t w = threadIdx.x >> 6, lane = __lane_id();
  for (uint32_t shift = 0; shift < nbits; shift += 8) {
    for (int i = threadIdx.x; i < 4 * 256 / 2; i += kT) reinterpret_cast<uint32_t*>(&S.hist[0][0])[i] = 0;
    __syncthreads();
    uint32_t dig[kWaveSpan / 64], loc[kWaveSpan / 64];
#pragma unroll
    for (int j = 0; j < (int)(kWaveSpan / 64); j++) {
      const uint32_t e = w * kWaveSpan + j * 64 + lane;
      const bool act = e < n;
      const uint64_t amask = __ballot(act);
      uint32_t d = act ? (kin[e] >> shift) & 255u : 0u;
      const uint64_t peers = match_byte(d, amask);
      const uint32_t rank = __popcll(peers & lanemask_lt());
      uint32_t old = act ? S.hist[w][d] : 0u;
      const bool leader = act && ((peers & lanemask_lt()) == 0);
      if (leader) S.hist[w][d] = (uint16_t)(old + (uint32_t)__popcll(peers));
      dig[j] = d;
      loc[j] = old + rank;
    }
    __syncthreads();
    {  // digit bases: exclusive over (digit, wave)
      const uint32_t d = threadIdx.x;
      uint32_t c0 = S.hist[0][d], c1 = S.hist[1][d], c2 = S.hist[2][d], c3 = S.hist[3][d];
      uint32_t tot = c0 + c1 + c2 + c3;
      uint32_t incl = block_incl_sum(tot, S.sh, (uint32_t*)nullptr);
      uint32_t b = incl - tot;
      S.hist[0][d] = (uint16_t)b;
      S.hist[1][d] = (uint16_t)(b + c0);
      S.hist[2][d] = (uint16_t)(b + c0 + c1);
      S.hist[3][d] = (uint16_t)(b + c0 + c1 + c2);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < (int)(kWaveSpan / 64); j++) {
      const uint32_t e = w * kWaveSpan + j * 64 + lane;
      if (e < n) {
        const uint32_t dst = S.hist[w][dig[j]] + loc[j];
        kout[dst] = kin[e];
        vout[dst] = vin[e];
      }
    }
    __syncthreads();
    uint32_t* t;
    t = kin; kin = kout; kout = t;
    t = vin; vin = vout; vout = t;
  }
  keys = kin;
  vals = vin;
}

// Diagnostic stamps (BZG_DEBUG builds only): phase durations summed over workgroups.
#define STAMP(k)                                                                    \
  if constexpr (kStamp) {                                                           \
    __syncthreads();                                                                \
    if (threadIdx.x == 0) {                                                         \
      const uint64_t now = __builtin_amdgcn_s_memtime();                            \
      atomicAdd((unsigned long long*)&stamps[k], (unsigned long long)(now - t_last)); \
      t_last = now;                                                                 \
    }                                                                               \
  }

template <bool kStamp>
__global__ void __launch_bounds__(kT) BZG_SGPR_LIMIT k_tile_sort(const Grp* __restrict__ small, uint32_t n_small,
                                                  const uint32_t* __restrict__ first, const uint32_t* __restrict__ last,
                                                  uint32_t key_bits, SortBufs B, Grp* __restrict__ next,
                                                  uint32_t* __restrict__ n_next, bool isa_valid,
                                                  uint64_t* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  TileLds& S = *reinterpret_cast<TileLds*>(smem);
  const uint32_t t = blockIdx.x;
  const uint32_t i0 = first[t];
  if (i0 == 0xffffffffu) return;
  uint64_t t_last = kStamp ? __builtin_amdgcn_s_memtime() : 0;
  // items of this tile: i0 .. i1-1 with P[i]/kWin == t (at most kWin/2: items hold >= 2 elements)
  const uint32_t i1 = min(last[t], i0 + kWin / 2);
  const uint32_t ni = i1 - i0;
  // Items larger than kSmall (sorted by the digit passes) are compacted away: their
  // tile-local size is 0.  Offsets are recomputed over the kept items.
  for (uint32_t j = threadIdx.x; j < ni; j += kT) {
    const Grp g = small[i0 + j];
    S.istart[j] = g.start;
    S.iunit[j] = g.unit | ((g.flags & 1u) << 31);
    S.ioff[j] = g.size <= kSmall ? g.size : 0u;
  }
  __syncthreads();
  uint32_t my_sz[kWin / 2 / kT + 1];
  uint32_t my_sum = 0;
#pragma unroll
  for (int q = 0; q < (int)(kWin / 2 / kT + 1); q++) {
    const uint32_t j = threadIdx.x * (kWin / 2 / kT + 1) + q;
    const uint32_t sz = j < ni ? S.ioff[j] : 0u;
    my_sz[q] = sz;
    my_sum += sz;
  }
  {
    uint32_t tot_e;
    const uint32_t incl = block_incl_sum(my_sum, S.sh, &tot_e);
    uint32_t o = incl - my_sum;
#pragma unroll
    for (int q = 0; q < (int)(kWin / 2 / kT + 1); q++) {
      const uint32_t j = threadIdx.x * (kWin / 2 / kT + 1) + q;
      if (j < ni) S.ioff[j] = o;
      o += my_sz[q];
    }
    if (threadIdx.x == 0) S.ioff[ni] = tot_e;
  }
  __syncthreads();
  const uint32_t n = S.ioff[ni];
  if (n == 0) return;
  STAMP(0);
  const uint32_t kmask = key_bits >= 32 ? 0xffffffffu : ((1u << key_bits) - 1u);
  {  // owner map: item index of every element (mark item starts, then a block max-scan)
    uint32_t* owner = S.keyB;
    uint4* o4 = reinterpret_cast<uint4*>(owner);
    for (uint32_t i = threadIdx.x; i < kTileCap / 4; i += kT) o4[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < ni; j += kT)
      if (S.ioff[j + 1] > S.ioff[j]) owner[S.ioff[j]] = j;
    __syncthreads();
    uint4 q4[kPer / 4];
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < (int)(kPer / 4); q++) {
      q4[q] = o4[threadIdx.x * (kPer / 4) + q];
      m = max(m, max(max(q4[q].x, q4[q].y), max(q4[q].z, q4[q].w)));
    }
    const uint32_t incl = block_incl_max(m, S.sh);
    uint32_t run = __shfl_up(incl, 1);
    if (__lane_id() == 0) run = threadIdx.x >= 64 ? S.sh[(threadIdx.x >> 6) - 1] : 0u;
    if (threadIdx.x == 0) run = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < (int)(kPer / 4); q++) {
      q4[q].x = run = max(run, q4[q].x);
      q4[q].y = run = max(run, q4[q].y);
      q4[q].z = run = max(run, q4[q].z);
      q4[q].w = run = max(run, q4[q].w);
      o4[threadIdx.x * (kPer / 4) + q] = q4[q];
    }
    __syncthreads();
  }
  for (uint32_t e = threadIdx.x; e < n; e += kT) {
    const uint32_t lo = S.keyB[e];
    const uint32_t s = S.istart[lo] + (e - S.ioff[lo]);
    const bool alt = S.iunit[lo] >> 31;
    const uint32_t k = alt ? B.key2[s] : B.key[s];
    const uint32_t v = alt ? B.sa2[s] : B.sa[s];
    S.keyA[e] = (lo << key_bits) | (k & kmask);
    S.valA[e] = v;
  }
  __syncthreads();
  STAMP(1);
  const uint32_t item_bits = 32 - __builtin_clz(ni);  // ni >= 1
  // largest item in the tile decides the method
  {
    uint32_t mx = 0;
    for (uint32_t j = threadIdx.x; j < ni; j += kT) mx = max(mx, S.ioff[j + 1] - S.ioff[j]);
    mx = block_incl_max(mx, S.sh);
    if (threadIdx.x == kT - 1) S.misc[3] = mx;
    __syncthreads();
  }
  uint32_t *keys, *vals;
  if (S.misc[3] <= kRankMax) {
    // rank counting: element e goes to ioff[item] + #{f in item : (key_f, f) < (key_e, e)};
    // lanes of one item read the same key at each step (LDS broadcast)
    for (uint32_t e = threadIdx.x; e < n; e += kT) {
      const uint32_t ke = S.keyA[e];
      const uint32_t item = ke >> key_bits;
      const uint32_t lo = S.ioff[item], hi = S.ioff[item + 1];
      uint32_t r = 0;
      for (uint32_t f = lo; f < hi; f++) {
        const uint32_t kf = S.keyA[f];
        r += (kf < ke) | ((kf == ke) & (f < e));
      }
      S.keyB[lo + r] = ke;
      S.valB[lo + r] = S.valA[e];
    }
    __syncthreads();
    keys = S.keyB;
    vals = S.valB;
    STAMP(2);
  } else {
    lds_radix_sort(S, n, key_bits + item_bits, keys, vals);
    STAMP(3);
  }
  // group detection over the sorted composite keys; thread t owns [kPer*t, kPer*t + kPer)
  const uint32_t e0 = threadIdx.x * kPer;
  uint32_t kq[kPer];
#pragma unroll
  for (int q = 0; q < (int)(kPer / 4); q++) {
    const uint4 a = reinterpret_cast<const uint4*>(keys + e0)[q];
    kq[4 * q] = a.x; kq[4 * q + 1] = a.y; kq[4 * q + 2] = a.z; kq[4 * q + 3] = a.w;
  }
  uint32_t smask = 0;  // bit q: element e0 + q starts a group
  {
    uint32_t prev = (e0 > 0 && e0 <= n) ? keys[e0 - 1] : 0u;
#pragma unroll
    for (int q = 0; q < (int)kPer; q++) {
      const uint32_t e = e0 + q;
      if (e < n && (e == 0 || kq[q] != prev)) smask |= 1u << q;
      prev = kq[q];
    }
  }
  const uint32_t starts = __popc(smask);
  uint32_t ngroups;
  const uint32_t incl = block_incl_sum(starts, S.sh, &ngroups);
  // gpos[o] = first element of group o (free key buffer); gid[e] = group of e (free val buffer)
  uint32_t* gpos = (keys == S.keyA) ? S.keyB : S.keyA;
  uint32_t* gid = (vals == S.valA) ? S.valB : S.valA;
  {
    uint32_t o = incl - starts;
    uint32_t gq[kPer];
#pragma unroll
    for (int q = 0; q < (int)kPer; q++) {
      if ((smask >> q) & 1u) gpos[o++] = e0 + q;
      gq[q] = o - 1;  // unused for e >= n
    }
#pragma unroll
    for (int q = 0; q < (int)(kPer / 4); q++)
      reinterpret_cast<uint4*>(gid + e0)[q] = make_uint4(gq[4 * q], gq[4 * q + 1], gq[4 * q + 2], gq[4 * q + 3]);
  }
  if (threadIdx.x == 0) gpos[ngroups] = n;
  __syncthreads();
  STAMP(4);
  // groups of size >= 2 go to the next iteration
  uint32_t nnew = 0;
  {
    uint32_t o = incl - starts;
    for (uint32_t m = smask; m; m &= m - 1, o++) nnew += (gpos[o + 1] - (e0 + __builtin_ctz(m)) >= 2);
  }
  uint32_t tot_new;
  const uint32_t incl_new = block_incl_sum(nnew, S.sh, &tot_new);
  if (threadIdx.x == 0) S.misc[1] = tot_new ? atomicAdd(n_next, tot_new) : 0;
  __syncthreads();
  if (nnew) {
    uint32_t wpos = S.misc[1] + incl_new - nnew;
    uint32_t o = incl - starts;
    for (uint32_t m = smask; m; m &= m - 1, o++) {
      const uint32_t e = e0 + __builtin_ctz(m);
      const uint32_t sz = gpos[o + 1] - e;
      if (sz >= 2) {
        const uint32_t item = kq[__builtin_ctz(m)] >> key_bits;
        next[wpos++] = Grp{S.istart[item] - S.ioff[item] + e, sz, S.iunit[item] & 0x7fffffffu, 0};
      }
    }
  }
  // element-parallel output: SA in slot order (coalesced); an ISA entry is rewritten only
  // when the rank changes (isa_valid: every member's ISA already holds its item's start)
  for (uint32_t e = threadIdx.x; e < n; e += kT) {
    const uint32_t item = keys[e] >> key_bits;
    const uint32_t istart = S.istart[item];
    const uint32_t base = istart - S.ioff[item];
    const uint32_t v = vals[e];
    B.sa[base + e] = v;
    const uint32_t gslot = base + gpos[gid[e]];
    if (!isa_valid || gslot != istart) B.isa[B.units[S.iunit[item] & 0x7fffffffu].sbase + v] = gslot;
  }
  STAMP(5);
  if constexpr (kStamp) {
    if (threadIdx.x == 0) atomicAdd((unsigned long long*)&stamps[6], 1ull);
    if (threadIdx.x == 0) atomicAdd((unsigned long long*)&stamps[7], (unsigned long long)n);
  }
}

// Equal-key groups larger than kSmall: everyone gets the bucket start as rank.
__global__ void __launch_bounds__(kT) k_equal(const Grp* __restrict__ G, uint32_t nG, const uint32_t* __restrict__ TP,
                                              SortBufs B, Grp* __restrict__ next, uint32_t* __restrict__ n_next) {
  const uint32_t t = blockIdx.x;
  const uint32_t g = upper_idx(TP, nG, t);
  const Grp gr = G[g];
  const uint32_t c = t - TP[g];
  const uint32_t lo = c * kDTile, hi = min(gr.size, lo + kDTile);
  const uint32_t sb = B.units[gr.unit].sbase;
  const uint32_t* vs = (gr.flags & 1) ? B.sa2 : B.sa;
  for (uint32_t e = lo + threadIdx.x; e < hi; e += kT) {
    const uint32_t v = vs[gr.start + e];
    B.sa[gr.start + e] = v;
    B.isa[sb + v] = gr.start;
  }
  if (c == 0 && threadIdx.x == 0) next[atomicAdd(n_next, 1u)] = Grp{gr.start, gr.size, gr.unit, 0};
}

}  // namespace

// ------------------------------------------------------------------------------------
void doubling_sort(Workspace& ws, const SortBufs& B, const Grp* L0, uint32_t nL0, uint32_t h, int* iterations,
                   uint64_t* revisited, hipStream_t st) {
  if (nL0 == 0) return;
  // element total of the initial list bounds every later list (summed on the device)
  uint64_t T = 0;
  {
    uint32_t* sz = ws.u32("dbl_P", (size_t)nL0 + 16);
    uint32_t* tot0 = ws.u32("dbl_T0", 16);
    uint32_t* scr = ws.u32z("dbl_scan", scan_scratch_words((size_t)nL0 + 16) + 64);
    k_group_sizes<<<(unsigned)ceil_div64(nL0, kT), kT, 0, st>>>(L0, nL0, sz);
    HIP_OK(hipGetLastError());
    scan_u32(ScanOp::Sum, true, sz, sz, nL0, tot0, scr, st);
    uint32_t t32 = 0;
    ws.read_small(&t32, tot0, 4, st);
    T = t32;
  }
  const size_t lcap = T / 2 + nL0 + 16;
  const size_t bigcap = T / kSmall + nL0 + 16;
  Grp* L = ws.typed<Grp>("dbl_L", lcap);
  Grp* Ln = ws.typed<Grp>("dbl_Ln", lcap);
  Grp* small = ws.typed<Grp>("dbl_small", lcap);
  Grp* large = ws.typed<Grp>("dbl_large", bigcap);
  Grp* large2 = ws.typed<Grp>("dbl_large2", bigcap);
  Grp* equal = ws.typed<Grp>("dbl_equal", bigcap);
  uint32_t* P = ws.u32("dbl_P", lcap + 16);
  const size_t max_dtiles = T / kDTile + bigcap + 16;
  uint32_t* TP = ws.u32("dbl_TP", max_dtiles + 16);
  uint32_t* first = ws.u32("dbl_first", T / kWin + 64);
  uint32_t* last = ws.u32("dbl_last", T / kWin + 64);
  uint32_t* gmap = ws.u32("dbl_gmap", T + 16);
  uint32_t* hist = ws.u32("dbl_hist", max_dtiles * 256);
  uint32_t* tot = ws.u32("dbl_tot", bigcap * 256);
  uint32_t* cnt = ws.u32("dbl_cnt", 64);
  uint32_t* scratch = ws.u32z("dbl_scan", scan_scratch_words(std::max<size_t>(std::max<size_t>(lcap, max_dtiles), T + 16)) + 64);
  HIP_OK(hipMemcpyAsync(L, L0, sizeof(Grp) * nL0, hipMemcpyDeviceToDevice, st));
  // counters: 0 total(scan), 1 n_large, 2 n_small, 3 n_next(L'), 4 n_large2, 5 n_equal, 6 tiles
  uint32_t hc[8];
  auto read_counters = [&]() { ws.read_small(hc, cnt, sizeof(hc), st); };
  auto grid = [](uint64_t n) { return (unsigned)std::max<uint64_t>(1, ceil_div64(n, kT)); };
  const size_t tile_lds = sizeof(TileLds);
  static_assert(4 * sizeof(TileLds) <= 160 * 1024, "four tile-sort workgroups must fit one CU's LDS");
  static bool attr_set = false;
  if (!attr_set) {
    HIP_OK(hipFuncSetAttribute((const void*)k_tile_sort<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tile_lds));
    attr_set = true;
  }
  uint32_t nL = nL0;
  int iters = 0;
  while (nL > 0) {
    ++iters;
    k_group_sizes<<<grid(nL), kT, 0, st>>>(L, nL, P);
    HIP_OK(hipGetLastError());
    scan_u32(ScanOp::Sum, true, P, P, nL, cnt + 0, scratch, st);
    HIP_OK(hipMemsetAsync(cnt + 1, 0, 7 * 4, st));
    read_counters();
    const uint32_t totalL = hc[0];
    if (revisited) *revisited += totalL;
    static const bool debug = getenv("BZG_DEBUG") != nullptr;
    if (debug) fprintf(stderr, "[bzg sort S3] iter %d: h=%u groups=%u elems=%u\n", iters, h, nL, totalL);
    HIP_OK(hipMemsetAsync(gmap, 0, (size_t)totalL * 4, st));
    k_mark_groups<<<grid(nL), kT, 0, st>>>(P, nL, gmap);
    HIP_OK(hipGetLastError());
    scan_u32(ScanOp::Max, false, gmap, gmap, totalL, cnt + 7, scratch, st);
    k_gather<<<grid(totalL), kT, 0, st>>>(L, P, gmap, totalL, h, B);
    HIP_OK(hipGetLastError());
    k_extract_large<<<grid(nL), kT, 0, st>>>(L, nL, 0, large, cnt + 1);
    HIP_OK(hipGetLastError());
    read_counters();
    uint32_t n_large = hc[1];
    static const uint32_t digs[3] = {12, 4, 0};
    const int ndig = 3;
    Grp* lg = large;
    Grp* lg2 = large2;
    for (int di = 0; di < ndig && n_large > 0; di++) {
      const int mode = di == ndig - 1 ? 2 : 0;
      k_group_tiles<<<grid(n_large), kT, 0, st>>>(lg, n_large, TP);
      HIP_OK(hipGetLastError());
      scan_u32(ScanOp::Sum, true, TP, TP, n_large, cnt + 6, scratch, st);
      HIP_OK(hipMemsetAsync(cnt + 4, 0, 4, st));
      read_counters();
      const uint32_t ntiles = hc[6];
      k_dhist<<<ntiles, kT, 0, st>>>(lg, n_large, TP, digs[di], B, hist);
      HIP_OK(hipGetLastError());
      k_doff<<<n_large, kT, 0, st>>>(lg, n_large, TP, hist, tot, mode, small, cnt + 2, lg2, cnt + 4, equal, cnt + 5);
      HIP_OK(hipGetLastError());
      k_dscatter<<<ntiles, kT, 0, st>>>(lg, n_large, TP, digs[di], B, hist, tot);
      HIP_OK(hipGetLastError());
      k_dsingle<<<ntiles, kT, 0, st>>>(lg, n_large, TP, B, tot);
      HIP_OK(hipGetLastError());
      read_counters();
      n_large = hc[4];
      std::swap(lg, lg2);
    }
    // (cnt + 3, the next list's count, was cleared with cnt + 1..7 at the top of the iteration:
    // only k_tile_sort and k_equal below append to it)
    const uint32_t kbits = 20u;
    {  // groups of L small enough for LDS: tiles straight over L (P still holds L's prefix)
      const uint32_t ntiles = ceil_div(totalL, kWin);
      k_tile_first<<<grid(nL), kT, 0, st>>>(P, nL, ntiles, first, last);
      HIP_OK(hipGetLastError());
      k_tile_sort<false><<<ntiles, kT, tile_lds, st>>>(L, nL, first, last, kbits, B, Ln, cnt + 3, true, nullptr);
      HIP_OK(hipGetLastError());
    }
    read_counters();
    const uint32_t n_small = hc[2];
    const uint32_t n_equal = hc[5];
    if (n_small > 0) {  // buckets emitted by the digit passes
      k_group_sizes<<<grid(n_small), kT, 0, st>>>(small, n_small, P);
      HIP_OK(hipGetLastError());
      scan_u32(ScanOp::Sum, true, P, P, n_small, cnt + 0, scratch, st);
      read_counters();
      const uint32_t tot_small = hc[0];
      const uint32_t ntiles = ceil_div(tot_small, kWin);
      k_tile_first<<<grid(n_small), kT, 0, st>>>(P, n_small, ntiles, first, last);
      HIP_OK(hipGetLastError());
      k_tile_sort<false><<<ntiles, kT, tile_lds, st>>>(small, n_small, first, last, kbits, B, Ln, cnt + 3, false, nullptr);
      HIP_OK(hipGetLastError());
    }
    if (n_equal > 0) {
      k_group_tiles<<<grid(n_equal), kT, 0, st>>>(equal, n_equal, TP);
      HIP_OK(hipGetLastError());
      scan_u32(ScanOp::Sum, true, TP, TP, n_equal, cnt + 6, scratch, st);
      read_counters();
      k_equal<<<hc[6], kT, 0, st>>>(equal, n_equal, TP, B, Ln, cnt + 3);
      HIP_OK(hipGetLastError());
    }
    if (n_small > 0 || n_equal > 0) read_counters();  // (else hc[3] is already the count)
    nL = hc[3];
    std::swap(L, Ln);
    h *= 2;
    if (iters > 40) throw HipFailure(hipErrorUnknown);  // cannot happen for aperiodic roots
  }
  if (iterations) *iterations += iters;
}

}  // namespace bzg
