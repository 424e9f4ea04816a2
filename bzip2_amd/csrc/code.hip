// code.hip -- stages A7/A8/A3: coding-table optimisation, Huffman code lengths, canonical
// codes, bit accounting and bit packing of every block, plus stream framing.
//
// Reference: sendMTFValues (compress.c:250-818), BZ2_hbMakeCodeLengths / BZ2_hbAssignCodes
// (huffman.c:63-166), BZ2_compressBlock framing (compress.c:822-881).  One workgroup owns one
// block for the table passes; selector groups of 50 symbols are costed in parallel and their
// per-table symbol frequencies gathered with LDS atomics; each table's heap Huffman runs on
// one lane with the reference's exact tie order.  Packing computes every field's bit offset
// with block-level scans and ORs 32-bit big-endian words into the (zeroed) output.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "stages.h"
#include "scan.h"

namespace bzg {

namespace {
constexpr int kT = 256;

// BZ2_hbMakeCodeLengths (huffman.c:63-148), called by all 64 lanes of a wave.  Leaf weight =
// max(freq,1) << 8 | 0, merge = sum of weights | (1 + max depth); heap moves use strict '<' on
// weights only; rescale with w = 1 + w/2 while any length exceeds max_len.
// The heap itself is sequential and runs on lane 0.  Heap entries carry their weight
// (weight << 32 | node), so a DOWNHEAP level is one 16-byte read of the two children, and
// UPHEAP reads one parent per level.  A heap wave is as much issue-bound as latency-bound:
// loading two or three levels ahead (and three ancestors at once) cost more in selects than it
// saved in round trips (profiles/r06_ab_heap_lookahead.txt: one heap 545 -> 415 us at 258
// symbols).  Lengths (parent-chain walks) and the rescale run on all lanes.
constexpr int kHeapCap = kMaxAlpha + 14;  // 272 entries (the 16-byte child reads stay inside)
__device__ __forceinline__ int32_t hb_wt(uint64_t e) { return (int32_t)(e >> 32); }

__device__ __forceinline__ void hb_sift_up(uint64_t* heap, int z, uint64_t item) {
  while (hb_wt(item) < hb_wt(heap[z >> 1])) {  // heap[0]: the weight-0 sentinel stops at the root
    heap[z] = heap[z >> 1];
    z >>= 1;
  }
  heap[z] = item;
}

// The reference's DOWNHEAP (huffman.c:46-59): at each level the smaller child (the right one
// only when strictly smaller) moves up unless item is strictly lighter.
__device__ __forceinline__ void hb_sift_down(uint64_t* heap, int nheap, uint64_t item) {
  const uint4* h4 = reinterpret_cast<const uint4*>(heap);  // h4[z] = heap[2z], heap[2z + 1]
  int z = 1;
  for (;;) {
    const int y = 2 * z;
    if (y > nheap) break;
    const uint4 q = h4[z];
    uint64_t c = ((uint64_t)q.y << 32) | q.x;
    int k = 0;
    if (y < nheap && (int32_t)q.w < (int32_t)q.y) {
      c = ((uint64_t)q.w << 32) | q.z;
      k = 1;
    }
    if (hb_wt(item) < hb_wt(c)) break;
    heap[z] = c;
    z = y + k;
  }
  heap[z] = item;
}

// `rescales`: leaf weights halved that many times before the first round (the weights of
// round 1 + rescales); at most kRounds rounds.  Returns whether the lengths fit max_len.
template <int kRounds>
__device__ bool hb_code_lengths(uint8_t* len, const uint32_t* freq, int alpha, int max_len, uint64_t* heap,
                                int32_t* weight, int32_t* parent, int rescales) {
  const int lane = (int)__lane_id();
  for (int i = lane; i < alpha; i += 64) {
    uint32_t f = freq[i] == 0 ? 1u : freq[i];
    for (int k = 0; k < rescales; k++) f = 1 + f / 2;
    weight[i + 1] = (int32_t)(f << 8);
  }
  for (int round = 0; round < kRounds; round++) {  // converges in a few rounds for valid tables
    for (int i = lane; i < 2 * alpha; i += 64) parent[i] = -1;
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      int nodes = alpha, nheap = 0;
      heap[0] = 0;  // weight 0 sentinel above the root
      for (int i = 1; i <= alpha; i++) hb_sift_up(heap, ++nheap, ((uint64_t)(uint32_t)weight[i] << 32) | (uint32_t)i);
      while (nheap > 1) {
        uint64_t pick[2];
        for (int k = 0; k < 2; k++) {
          pick[k] = heap[1];
          const uint64_t item = heap[nheap--];
          hb_sift_down(heap, nheap, item);
        }
        nodes++;
        parent[(uint32_t)pick[0]] = parent[(uint32_t)pick[1]] = nodes;
        const int32_t w0 = hb_wt(pick[0]), w1 = hb_wt(pick[1]);
        const int32_t d0 = w0 & 0xff, d1 = w1 & 0xff;
        const int32_t wn = (int32_t)(((uint32_t)w0 & 0xffffff00u) + ((uint32_t)w1 & 0xffffff00u)) | (1 + (d0 > d1 ? d0 : d1));
        hb_sift_up(heap, ++nheap, ((uint64_t)(uint32_t)wn << 32) | (uint32_t)nodes);
      }
    }
    __builtin_amdgcn_wave_barrier();
    bool too_long = false;
    for (int i = lane + 1; i <= alpha; i += 64) {
      int d = 0, k = i;
      while (parent[k] >= 0) {
        k = parent[k];
        d++;
      }
      len[i - 1] = (uint8_t)d;
      if (d > max_len) too_long = true;
    }
    if (__ballot(too_long) == 0) return true;
    for (int i = lane + 1; i <= alpha; i += 64) weight[i] = (1 + ((weight[i] >> 8) / 2)) << 8;
  }
  return false;
}

struct HuffLds {  // one wave's table
  alignas(16) uint64_t heap[kHeapCap];
  int32_t weight[kMaxAlpha + 2];
  int32_t parent[kMaxAlpha * 2];
  uint32_t fq[kMaxAlpha];
  uint8_t len[kMaxAlpha + 2];
  uint32_t word;
};

// Rounds 1 and 2 of one table at once (k_huff_spec): workgroup r0 of the table runs round
// 1 + r0 alone (its leaf weights halved r0 times: a round's weights depend only on the
// frequencies, not on the previous round's tree).  Round 1's lengths, when they fit, go
// straight to L; round 2's to the table's scratch.  The second workgroup to finish (one
// atomic on the table's word: finish count in bits 0-1, "round 1 + r0 fits" in bit 2 + r0)
// keeps the first round that fits -- or, when neither does, goes on from round 3 -- and
// resets the word (and the frequencies, when `rf`).  The same lengths as the reference's
// rounds one after another (huffman.c:63-148).  A table that needs one rescale (22 of 2,688
// on the 100 MB bench text, in 6 of its 8 launches) then costs one round of latency instead
// of two; but the round-1 waves run slower beside the round-2 ones (a launch of 336 tables:
// 115-135 us for one round alone, 175-200 with the speculation, 210-225 for two rounds), so
// the gain is 60-80 us per 100 MB call (profiles/r06_ab_huff_spec.txt).
__device__ void hb_spec_table(HuffLds& S, int alpha, int max_len, uint32_t r0, uint32_t* word, uint8_t* scratch,
                              uint8_t* L, uint32_t* rf) {
  const bool ok = hb_code_lengths<1>(S.len, S.fq, alpha, max_len, S.heap, S.weight, S.parent, (int)r0);
  if (ok) {
    uint8_t* dst = r0 == 0 ? L : scratch;
    for (int v = threadIdx.x; v < alpha; v += 64) dst[v] = S.len[v];
  }
  const uint32_t mine = 1u | ((ok ? 1u : 0u) << (2 + r0));
  if (threadIdx.x == 0) {
    __threadfence();  // the lengths before the count
    S.word = atomicAdd(word, mine) + mine;
    __threadfence();
  }
  __syncthreads();
  const uint32_t w = S.word;
  if ((w & 3u) != 2u) return;  // the other workgroup finishes the table
  if (!(w & 4u)) {
    const uint8_t* src = S.len;
    if (w & 8u) {
      if (r0 == 0) src = scratch;  // round 2 ran in the other workgroup
    } else {
      (void)hb_code_lengths<62>(S.len, S.fq, alpha, max_len, S.heap, S.weight, S.parent, 2);
    }
    for (int v = threadIdx.x; v < alpha; v += 64) L[v] = src[v];
  }
  if (rf)
    for (int v = threadIdx.x; v < alpha; v += 64) rf[v] = 0;  // ready for the next iteration
  if (threadIdx.x == 0) *word = 0;
}

// The same BZ2_hbMakeCodeLengths run by one lane per table, kHuffLanes tables per wave, for
// launches with many tables (the single-lane heap issues every instruction for the whole wave:
// with thousands of tables per launch, BASELINE config 5, k_huff is VALU-bound, not
// latency-bound).  Each lane keeps its table in its own LDS region (heap entries carrying
// their weight, leaf weights, parents, depths) and runs the reference's loops as written:
// UPHEAP / DOWNHEAP with strict '<' on weights, the rescale rounds, lengths as depths (nodes
// are created in increasing order, so the depths fill top-down in one pass).
constexpr int kHuffLanes = 8;
struct HuffLane {  // 3,108 bytes: 8 lanes' regions in 24.9 KB, 6 workgroups per CU
  uint64_t heap[kMaxAlpha + 1];
  int16_t parent[2 * kMaxAlpha];  // then each node's depth, in place
  uint32_t pad;                   // (regions of different lanes start in different banks)
};
// The leaf weights live in the table's frequency words in global memory (read at the start,
// touched again only by a rescale), which are zeroed at the end when `reset` (ready for the
// next iteration's counts).
__device__ void hb_lane_lengths(HuffLane& H, uint32_t* __restrict__ wt, bool reset, int alpha, int max_len,
                                uint8_t* __restrict__ lens) {
  for (int i = 0; i < alpha; i++) {
    const uint32_t f = wt[i];
    wt[i] = (f == 0 ? 1u : f) << 8;
  }
  for (int round = 0; round < 64; round++) {
    int nheap = 0, nodes = alpha;
    H.heap[0] = 0;  // weight 0 sentinel above the root
    for (int i = 1; i <= alpha; i++) {
      H.parent[i] = -1;
      const uint64_t tmp = ((uint64_t)wt[i - 1] << 32) | (uint32_t)i;
      int z = ++nheap;
      while (hb_wt(tmp) < hb_wt(H.heap[z >> 1])) {
        H.heap[z] = H.heap[z >> 1];
        z >>= 1;
      }
      H.heap[z] = tmp;
    }
    while (nheap > 1) {
      uint64_t pick[2];
      for (int k = 0; k < 2; k++) {
        pick[k] = H.heap[1];
        const uint64_t tmp = H.heap[nheap--];
        int z = 1;
        for (;;) {
          int y = z << 1;
          if (y > nheap) break;
          uint64_t c = H.heap[y];
          if (y < nheap) {
            const uint64_t c2 = H.heap[y + 1];
            if (hb_wt(c2) < hb_wt(c)) {
              c = c2;
              y++;
            }
          }
          if (hb_wt(tmp) < hb_wt(c)) break;
          H.heap[z] = c;
          z = y;
        }
        H.heap[z] = tmp;
      }
      nodes++;
      H.parent[(uint32_t)pick[0]] = H.parent[(uint32_t)pick[1]] = (int16_t)nodes;
      const int32_t w0 = hb_wt(pick[0]), w1 = hb_wt(pick[1]);
      const int32_t d0 = w0 & 0xff, d1 = w1 & 0xff;
      const int32_t wn = (int32_t)(((uint32_t)w0 & 0xffffff00u) + ((uint32_t)w1 & 0xffffff00u)) | (1 + (d0 > d1 ? d0 : d1));
      const uint64_t tmp = ((uint64_t)(uint32_t)wn << 32) | (uint32_t)nodes;
      int z = ++nheap;
      while (hb_wt(tmp) < hb_wt(H.heap[z >> 1])) {
        H.heap[z] = H.heap[z >> 1];
        z >>= 1;
      }
      H.heap[z] = tmp;
    }
    // depths top-down (a parent has a larger index than its children), in place of the parents
    H.parent[nodes] = 0;
    for (int k = nodes - 1; k >= 1; k--) H.parent[k] = (int16_t)(H.parent[H.parent[k]] + 1);
    bool too_long = false;
    for (int i = 1; i <= alpha; i++) {
      lens[i - 1] = (uint8_t)H.parent[i];
      too_long |= H.parent[i] > max_len;
    }
    if (!too_long) break;
    for (int i = 0; i < alpha; i++) wt[i] = (1 + ((wt[i] >> 8) / 2)) << 8;
  }
  if (reset)
    for (int i = 0; i < alpha; i++) wt[i] = 0;
}

__device__ __forceinline__ int n_groups(uint32_t nmtf) {  // compress.c:266-270
  return nmtf < 200 ? 2 : nmtf < 600 ? 3 : nmtf < 1200 ? 4 : nmtf < 2400 ? 5 : 6;
}

// ---- table optimisation (sendMTFValues, compress.c:250-561), one kernel per step:
//   k_init_tables: the initial contiguous partition (compress.c:276-319);
//   4 x { k_cf: cost of every 50-symbol group under each table, selection (lowest index wins
//          ties, compress.c:416-420) and per-table symbol frequencies -- several workgroups
//          per block, each over a slice of the groups;
//         k_huff: BZ2_hbMakeCodeLengths for every (block, table), one wave each };
//   k_cf (final mode): payload bits of every group under the final tables;
//   k_final: canonical codes, selector MTF, table and header bit counts.
// Workgroups per block in k_cf and k_pack (gridDim.x): at least kCfSlices (kPackSlices) and
// enough for about kSliceFill workgroups per launch, so that a call of few blocks (100 MB: 110
// blocks, 55 per k_cf half) is not a chain of steps on a hundred workgroups.
constexpr uint32_t kCfSlices = 2, kPackSlices = 1, kSliceMax = 8, kSliceFill = 768;
// tables per launch from which k_huff_lanes (a lane per table) replaces k_huff (a wave per
// table); BZG_HUFF_LANES_MIN overrides (A/B knob; 0 also routes the code-length test hook)
inline uint32_t huff_lanes_min() {
  static const uint32_t v = (uint32_t)std::max(0ll, env_ll("BZG_HUFF_LANES_MIN", 4096));
  return v;
}
// tables per launch up to which k_huff_spec tries rounds 1 and 2 at once (the launch's latency
// is its slowest table's; above it the extra waves cost throughput: code stage per call with
// and without, 336 tables per launch (100 MB): -0.23 ms, 834 (250 MB): -0.07 ms, 1,668
// (500 MB, measured with the round-5 heap): +1.0 ms, 3,336 (1 GB): +2 ms);
// BZG_HUFF_SPEC_MAX overrides (read per call: A/B knob, and 0 lets the code-length test take
// the one-round-at-a-time path)
inline uint32_t huff_spec_max() { return (uint32_t)std::max(0ll, env_ll("BZG_HUFF_SPEC_MAX", 1024)); }
inline uint32_t slices_for(uint32_t nb, uint32_t lo) {
  return std::max(lo, std::min(kSliceMax, ceil_div(kSliceFill, std::max(nb, 1u))));
}

__global__ void k_init_tables(uint32_t b0, const uint32_t* __restrict__ nmtf_g, const uint32_t* __restrict__ freq_g,
                              const uint32_t* __restrict__ ninuse, uint8_t* __restrict__ lens_g,
                              uint32_t* __restrict__ rf_g) {
  const uint32_t b = b0 + blockIdx.x;
  uint8_t* L = lens_g + (size_t)b * kNGroups * kMaxAlpha;
  for (int i = threadIdx.x; i < kNGroups * kMaxAlpha; i += blockDim.x) {
    L[i] = 0;
    rf_g[(size_t)b * kNGroups * kMaxAlpha + i] = 0;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const uint32_t nmtf = nmtf_g[b];
  const int alpha = (int)ninuse[b] + 2;
  const int ng = n_groups(nmtf);
  const uint32_t* freq = freq_g + (size_t)b * kMaxAlpha;
  for (int t = 0; t < ng; t++)
    for (int v = 0; v < alpha; v++) L[t * kMaxAlpha + v] = 15;
  int part = ng, rem = (int)nmtf, gs = 0;
  while (part > 0) {
    const int target = rem / part;
    int ge = gs - 1, acc = 0;
    while (acc < target && ge < alpha - 1) acc += (int)freq[++ge];
    if (ge > gs && part != ng && part != 1 && ((ng - part) % 2 == 1)) acc -= (int)freq[ge--];
    for (int v = gs; v <= ge; v++) L[(part - 1) * kMaxAlpha + v] = 0;
    part--;
    gs = ge + 1;
    rem -= acc;
  }
}

constexpr uint32_t kCfVec = (kT * kGroupSize + 8 * kT - 1) / (8 * kT);  // 16-byte words per thread per chunk
// One 64-bit length word per symbol (all six tables in 10-bit fields), so a symbol costs one
// LDS read and one add (two 32-bit words measured 0.4 ms per GB slower, round 4).
struct CfLds {
  alignas(16) uint16_t chunk[kT * kGroupSize + 8];
  uint64_t lenp[kMaxAlpha];
  uint32_t rfreq[kNGroups][kMaxAlpha * 2];  // 2 bank-spread copies per counter (thread & 1)
  uint32_t sh[8];
};
static_assert(kGroupSize * 17 < 1024, "a group's cost under one table fits a 10-bit field");

// final == 0: select tables and count frequencies (into rf_g); final == 1: payload bits of
// every group under its (already chosen) table into gbits_g, their sum into info_g[b*8+6].
__global__ void __launch_bounds__(kT) k_cf(uint32_t b0, const uint16_t* __restrict__ mtfv, const uint32_t* __restrict__ mtf_off,
                                           const uint32_t* __restrict__ nmtf_g, const uint8_t* __restrict__ lens_g,
                                           uint8_t* __restrict__ sel_g, uint32_t* __restrict__ rf_g,
                                           uint16_t* __restrict__ gbits_g, uint32_t* __restrict__ info_g, int final) {
  __shared__ CfLds S;
  const uint32_t b = b0 + blockIdx.y;
  const uint32_t nmtf = nmtf_g[b];
  const uint32_t nsel = ceil_div(nmtf, kGroupSize);
  const uint32_t nch = ceil_div(nsel, kT);
  const uint32_t cps = ceil_div(nch, gridDim.x);
  const uint32_t c0 = blockIdx.x * cps, c1 = min(nch, c0 + cps);
  if (c0 >= c1) return;
  const int ng = n_groups(nmtf);
  const uint16_t* mv = mtfv + mtf_off[b];
  const uint8_t* L = lens_g + (size_t)b * kNGroups * kMaxAlpha;
  for (int v = threadIdx.x; v < kMaxAlpha; v += kT) {
    uint64_t x = 0;
#pragma unroll
    for (int t = 0; t < kNGroups; t++) x |= (uint64_t)L[t * kMaxAlpha + v] << (10 * t);
    S.lenp[v] = x;
  }
  if (!final)
    for (int i = threadIdx.x; i < kNGroups * kMaxAlpha * 2; i += kT) (&S.rfreq[0][0])[i] = 0;
  uint8_t* selo = sel_g + (size_t)b * kMaxSelectors;
  uint32_t mybits = 0;
  // a chunk (kT groups) is read as 16-byte words (block offsets are multiples of 8 values);
  // the next chunk's words are loaded into registers while this one is costed
  uint4 q[kCfVec];
  auto load_chunk = [&](uint32_t ch) {
    const uint32_t lo = ch * kT * kGroupSize, hi = min(lo + kT * kGroupSize, nmtf);
#pragma unroll
    for (uint32_t k = 0; k < kCfVec; k++) {
      const uint32_t i = lo + 8 * (threadIdx.x + k * kT);
      q[k] = i < hi ? *reinterpret_cast<const uint4*>(mv + i) : make_uint4(0, 0, 0, 0);
    }
  };
  load_chunk(c0);
  for (uint32_t ch = c0; ch < c1; ch++) {
    const uint32_t g0 = ch * kT;
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kCfVec; k++) {
      const uint32_t j = 8 * (threadIdx.x + k * kT);
      if (j < kT * kGroupSize) *reinterpret_cast<uint4*>(S.chunk + j) = q[k];
    }
    if (ch + 1 < c1) load_chunk(ch + 1);
    __syncthreads();
    const uint32_t g = g0 + threadIdx.x;
    if (g < nsel) {
      // the group's 50 symbols in 25 registers, read as pairs (a group starts 100 bytes after the
      // last: 4-byte aligned, and 25 words apart keeps the lanes on distinct banks), once for
      // both the cost and the counting loops
      const uint32_t* cw = reinterpret_cast<const uint32_t*>(S.chunk + threadIdx.x * kGroupSize);
      const uint32_t n = min((uint32_t)kGroupSize, nmtf - g * kGroupSize);
      uint32_t sym[kGroupSize / 2];
#pragma unroll
      for (int k = 0; k < (int)kGroupSize / 2; k++) sym[k] = cw[k];
      auto sym_at = [&](int i) { return (sym[i >> 1] >> (16 * (i & 1))) & 0xffffu; };
      // 50 lengths <= 17: every 10-bit field sum stays below 1024
      uint64_t acc = 0;
      if (n == kGroupSize) {
#pragma unroll
        for (int i = 0; i < (int)kGroupSize; i++) acc += S.lenp[sym_at(i)];
      } else {
#pragma unroll
        for (int i = 0; i < (int)kGroupSize; i++)
          if ((uint32_t)i < n) acc += S.lenp[sym_at(i)];
      }
      uint32_t cost[kNGroups];
#pragma unroll
      for (int t = 0; t < kNGroups; t++) cost[t] = (uint32_t)(acc >> (10 * t)) & 1023u;
      if (final) {
        const uint32_t bits = cost[selo[g]];
        gbits_g[(size_t)b * kMaxSelectors + g] = (uint16_t)bits;
        mybits += bits;
      } else {
        int bt = 0;  // lowest index wins ties (compress.c:416-420)
        uint32_t bc = cost[0];
        for (int t = 1; t < ng; t++)
          if (cost[t] < bc) {
            bc = cost[t];
            bt = t;
          }
        selo[g] = (uint8_t)bt;
        // symbols 0..3 (RUNA, RUNB and the nearest ranks: most of the group on text) are
        // counted in registers first, so few lanes of a wave hit the same LDS counter
        // (four byte counters in one word: a group has at most 50 symbols)
        uint32_t f4 = 0;
        uint32_t* rfb = &S.rfreq[bt][threadIdx.x & 1u];
#pragma unroll
        for (int i = 0; i < (int)kGroupSize; i++) {
          const uint32_t v = sym_at(i);
          if ((uint32_t)i < n) {
            if (v > 3) atomicAdd(&rfb[v * 2], 1u);
            else f4 += 1u << (8 * v);
          }
        }
        const uint32_t f0 = f4 & 255u, f1 = (f4 >> 8) & 255u, f2 = (f4 >> 16) & 255u, f3 = f4 >> 24;
        if (f0) atomicAdd(&rfb[0], f0);
        if (f1) atomicAdd(&rfb[2], f1);
        if (f2) atomicAdd(&rfb[4], f2);
        if (f3) atomicAdd(&rfb[6], f3);
      }
    }
  }
  __syncthreads();
  if (final) {
    uint32_t tot;
    block_incl_sum(mybits, S.sh, &tot);
    if (threadIdx.x == 0) atomicAdd(&info_g[(size_t)b * 8 + 6], tot);
  } else {
    uint32_t* rf = rf_g + (size_t)b * kNGroups * kMaxAlpha;
    for (int i = threadIdx.x; i < ng * kMaxAlpha; i += kT) {
      const uint32_t v = (&S.rfreq[0][0])[2 * i] + (&S.rfreq[0][0])[2 * i + 1];
      if (v) atomicAdd(&rf[i], v);
    }
  }
}

// BZ2_hbMakeCodeLengths for table t of block b (one wave; the heap work is sequential).
__global__ void __launch_bounds__(64) k_huff(uint32_t b0, const uint32_t* __restrict__ nmtf_g, const uint32_t* __restrict__ ninuse,
                                             uint32_t* __restrict__ rf_g, uint8_t* __restrict__ lens_g) {
  __shared__ HuffLds S;
  const uint32_t b = b0 + blockIdx.x / kNGroups, t = blockIdx.x % kNGroups;
  const int ng = n_groups(nmtf_g[b]);
  if ((int)t >= ng) return;
  const int alpha = (int)ninuse[b] + 2;
  uint32_t* rf = rf_g + ((size_t)b * kNGroups + t) * kMaxAlpha;
  for (int v = threadIdx.x; v < alpha; v += 64) {
    S.fq[v] = rf[v];
    rf[v] = 0;  // ready for the next iteration
  }
  __syncthreads();
  (void)hb_code_lengths<64>(S.len, S.fq, alpha, kMaxCodeLen, S.heap, S.weight, S.parent, 0);
  __syncthreads();
  uint8_t* L = lens_g + ((size_t)b * kNGroups + t) * kMaxAlpha;
  for (int v = threadIdx.x; v < alpha; v += 64) L[v] = S.len[v];
}

// k_huff with rounds 1 and 2 of every table at once (hb_spec_table): workgroup g runs round
// 1 + g / nt of table g % nt of the launch's nt = n * kNGroups tables.
__global__ void __launch_bounds__(64) k_huff_spec(uint32_t b0, uint32_t nt, const uint32_t* __restrict__ nmtf_g,
                                                  const uint32_t* __restrict__ ninuse, uint32_t* __restrict__ rf_g,
                                                  uint8_t* __restrict__ lens_g, uint32_t* __restrict__ word_g,
                                                  uint8_t* __restrict__ scratch_g) {
  __shared__ HuffLds S;
  const uint32_t r0 = blockIdx.x >= nt ? 1u : 0u, tt = blockIdx.x - r0 * nt;
  const uint32_t b = b0 + tt / kNGroups, t = tt % kNGroups;
  if ((int)t >= n_groups(nmtf_g[b])) return;
  const int alpha = (int)ninuse[b] + 2;
  const size_t g = (size_t)b * kNGroups + t;
  uint32_t* rf = rf_g + g * kMaxAlpha;
  for (int v = threadIdx.x; v < alpha; v += 64) S.fq[v] = rf[v];
  __syncthreads();
  hb_spec_table(S, alpha, kMaxCodeLen, r0, word_g + g, scratch_g + g * kMaxAlpha, lens_g + g * kMaxAlpha, rf);
}

// k_huff with kHuffLanes tables per wave (one lane each): table tt = wave * kHuffLanes + lane of
// the launch's n blocks (tt / kNGroups, tt % kNGroups).
__global__ void __launch_bounds__(64) k_huff_lanes(uint32_t b0, uint32_t n, const uint32_t* __restrict__ nmtf_g,
                                                   const uint32_t* __restrict__ ninuse, uint32_t* __restrict__ rf_g,
                                                   uint8_t* __restrict__ lens_g) {
  __shared__ HuffLane H[kHuffLanes];
  const uint32_t lane = threadIdx.x, tt = blockIdx.x * kHuffLanes + lane;
  if (lane >= (uint32_t)kHuffLanes || tt >= n * kNGroups) return;
  const uint32_t b = b0 + tt / kNGroups, t = tt % kNGroups;
  if ((int)t >= n_groups(nmtf_g[b])) return;
  const int alpha = (int)ninuse[b] + 2;
  hb_lane_lengths(H[lane], rf_g + ((size_t)b * kNGroups + t) * kMaxAlpha, true, alpha, kMaxCodeLen,
                  lens_g + ((size_t)b * kNGroups + t) * kMaxAlpha);
}

// Test hooks: code lengths of n tables (freq[t * kMaxAlpha ..], alpha[t], max_len) with the
// same device routines as k_huff and k_huff_spec.
__global__ void __launch_bounds__(64) k_code_lengths_test(const uint32_t* __restrict__ freq_g,
                                                          const int32_t* __restrict__ alpha_g, int max_len,
                                                          uint8_t* __restrict__ lens_g) {
  __shared__ HuffLds S;
  const uint32_t t = blockIdx.x;
  const int alpha = alpha_g[t];
  for (int v = threadIdx.x; v < alpha; v += 64) S.fq[v] = freq_g[(size_t)t * kMaxAlpha + v];
  __syncthreads();
  (void)hb_code_lengths<64>(S.len, S.fq, alpha, max_len, S.heap, S.weight, S.parent, 0);
  __syncthreads();
  for (int v = threadIdx.x; v < alpha; v += 64) lens_g[(size_t)t * kMaxAlpha + v] = S.len[v];
}

__global__ void __launch_bounds__(64) k_code_lengths_spec(const uint32_t* __restrict__ freq_g,
                                                          const int32_t* __restrict__ alpha_g, uint32_t n, int max_len,
                                                          uint8_t* __restrict__ lens_g, uint32_t* __restrict__ word_g,
                                                          uint8_t* __restrict__ scratch_g) {
  __shared__ HuffLds S;
  const uint32_t r0 = blockIdx.x >= n ? 1u : 0u, t = blockIdx.x - r0 * n;
  const int alpha = alpha_g[t];
  for (int v = threadIdx.x; v < alpha; v += 64) S.fq[v] = freq_g[(size_t)t * kMaxAlpha + v];
  __syncthreads();
  hb_spec_table(S, alpha, max_len, r0, word_g + t, scratch_g + (size_t)t * kMaxAlpha, lens_g + (size_t)t * kMaxAlpha,
                nullptr);
}

__global__ void __launch_bounds__(64) k_code_lengths_lanes(const uint32_t* __restrict__ freq_g,
                                                           const int32_t* __restrict__ alpha_g, uint32_t n, int max_len,
                                                           uint8_t* __restrict__ lens_g) {
  __shared__ HuffLane H[kHuffLanes];
  const uint32_t lane = threadIdx.x, t = blockIdx.x * kHuffLanes + lane;
  if (lane >= (uint32_t)kHuffLanes || t >= n) return;
  hb_lane_lengths(H[lane], const_cast<uint32_t*>(freq_g) + (size_t)t * kMaxAlpha, false, alpha_g[t], max_len,
                  lens_g + (size_t)t * kMaxAlpha);
}

// Canonical codes (huffman.c:152-166), selector MTF (compress.c:573-631), table bits
// (compress.c:694-706) and the block's total bit count.  info_g[b*8+6] holds the payload bits.
__global__ void __launch_bounds__(kT) k_final(uint32_t b0, const uint32_t* __restrict__ nmtf_g, const uint32_t* __restrict__ ninuse,
                                              const uint32_t* __restrict__ inuse, const uint8_t* __restrict__ lens_g,
                                              uint32_t* __restrict__ codes_g, const uint8_t* __restrict__ sel_g,
                                              uint8_t* __restrict__ selmtf_g, uint32_t* __restrict__ info_g) {
  __shared__ uint8_t len[kNGroups][kMaxAlpha + 2];
  __shared__ uint8_t sel[kMaxSelectors + 4];
  __shared__ uint32_t sh[8];
  __shared__ uint32_t misc[16];
  const uint32_t b = b0 + blockIdx.x;
  const uint32_t nmtf = nmtf_g[b];
  const int alpha = (int)ninuse[b] + 2;
  const int ng = n_groups(nmtf);
  const uint32_t nsel = ceil_div(nmtf, kGroupSize);
  for (int i = threadIdx.x; i < kNGroups * kMaxAlpha; i += kT)
    len[i / kMaxAlpha][i % kMaxAlpha] = lens_g[(size_t)b * kNGroups * kMaxAlpha + i];
  for (uint32_t g = threadIdx.x; g < nsel; g += kT) sel[g] = sel_g[(size_t)b * kMaxSelectors + g];
  __syncthreads();
  // canonical codes (BZ2_hbAssignCodes, huffman.c:152-166), table t on wave t % 4 with all its
  // lanes: the code of symbol v is base[len v] + the number of symbols before v with the same
  // length, where base[min] = 0 and base[l + 1] = (base[l] + count[l]) << 1.  Symbols are taken
  // 64 at a time in index order; equal lengths inside a group of 64 are ranked by ballots, the
  // earlier groups through LDS counts.  (A serial lane-0 loop over 17 x 258 entries was about
  // 180 us of the tail of every call.)
  {
    __shared__ uint32_t lcnt[kT / 64][kMaxCodeLen + 2];
    __shared__ uint32_t lbase[kT / 64][kMaxCodeLen + 2];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    for (int t = (int)w; t < ng; t += kT / 64) {
      if (lane < kMaxCodeLen + 2) lcnt[w][lane] = 0;
      __builtin_amdgcn_wave_barrier();
      uint32_t rk[5], bits = 0;
      int mn = 32, mx = 0;
#pragma unroll
      for (int k = 0; k < 5; k++) {
        const int v = 64 * k + (int)lane;
        const bool in = v < alpha;
        const uint32_t l = in ? len[t][v] : 0u;
        uint64_t m = __ballot(in);
#pragma unroll
        for (int bit = 0; bit < 5; bit++) {
          const uint64_t bal = __ballot((l >> bit) & 1u);
          m &= ((l >> bit) & 1u) ? bal : ~bal;
        }
        rk[k] = in ? lcnt[w][l] + (uint32_t)__popcll(m & lanemask_lt()) : 0u;
        __builtin_amdgcn_wave_barrier();
        if (in && (m & lanemask_lt()) == 0) lcnt[w][l] += (uint32_t)__popcll(m);  // the first lane of each length
        __builtin_amdgcn_wave_barrier();
        if (in) {
          mn = min(mn, (int)l);
          mx = max(mx, (int)l);
          const int p = v == 0 ? (int)l : (int)len[t][v - 1];
          bits += 1 + 2 * (uint32_t)((int)l > p ? (int)l - p : p - (int)l);
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, __shfl_xor(mn, o, 64));
        mx = max(mx, __shfl_xor(mx, o, 64));
      }
      bits = wave_sum(bits);
      if (lane == 0) {
        uint32_t c = 0;
        for (int l = mn; l <= mx; l++) {
          lbase[w][l] = c;
          c = (c + lcnt[w][l]) << 1;
        }
        misc[8 + t] = bits + 5;
      }
      __builtin_amdgcn_wave_barrier();
      uint32_t* co = codes_g + ((size_t)b * kNGroups + t) * kMaxAlpha;
#pragma unroll
      for (int k = 0; k < 5; k++) {
        const int v = 64 * k + (int)lane;
        if (v < alpha) co[v] = lbase[w][len[t][v]] + rk[k];
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  // selector MTF in parallel: the MTF index of selector s at g is the number of tables used
  // more recently than s, where the initial order 0..5 counts as uses at times -1..-6.
  // Thread k owns a contiguous run of selectors; the last use of every table before the run
  // comes from a block max-scan.
  uint8_t* smo = selmtf_g + (size_t)b * kMaxSelectors;
  {
    const uint32_t per = ceil_div(nsel, (uint32_t)kT);
    const uint32_t g_lo = min(nsel, threadIdx.x * per), g_hi = min(nsel, g_lo + per);
    int32_t mine[kNGroups] = {-1, -1, -1, -1, -1, -1};  // last use inside my run (+1), 0 = none
    for (uint32_t g = g_lo; g < g_hi; g++) mine[sel[g]] = (int32_t)g + 1;
    int32_t lastu[kNGroups];
#pragma unroll
    for (int t = 0; t < kNGroups; t++) {
      const uint32_t m = mine[t] < 0 ? 0u : (uint32_t)mine[t];
      const uint32_t incl = block_incl_max(m, sh);
      uint32_t ex = __shfl_up(incl, 1);
      if (__lane_id() == 0) ex = threadIdx.x >= 64 ? sh[(threadIdx.x >> 6) - 1] : 0u;
      __syncthreads();
      lastu[t] = ex ? (int32_t)ex - 1 : -1 - t;
    }
    uint32_t sbits = 0;
    for (uint32_t g = g_lo; g < g_hi; g++) {
      const int s = sel[g];
      const int32_t ls = lastu[s];
      uint32_t j = 0;
#pragma unroll
      for (int t = 0; t < kNGroups; t++) j += lastu[t] > ls;
      lastu[s] = (int32_t)g;
      smo[g] = (uint8_t)j;
      sbits += j + 1;
    }
    uint32_t tot;
    block_incl_sum(sbits, sh, &tot);
    if (threadIdx.x == 0) misc[0] = tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t used16 = 0;
    for (int i = 0; i < 16; i++) {
      const uint32_t w = inuse[b * 8 + (i >> 1)];
      const uint32_t half = (i & 1) ? (w >> 16) : (w & 0xffffu);
      if (half) used16++;
    }
    uint32_t tbits = 0;
    for (int t = 0; t < ng; t++) tbits += misc[8 + t];
    uint32_t* info = info_g + (size_t)b * 8;
    const uint32_t data_bits = info[6];
    const uint32_t total = 48 + 32 + 1 + 24 + 16 + 16 * used16 + 3 + 15 + misc[0] + tbits + data_bits;
    info[0] = (uint32_t)ng;
    info[1] = nsel;
    info[2] = (uint32_t)alpha;
    info[3] = total;
    info[4] = misc[0];
    info[5] = tbits;
  }
}

// Bit offsets of every block, the combined CRC, the trailer position.
// Bit offset of every block and the running combined CRC (compress.c:826-828), continuing
// from the previous part of the batch: chain[0] = start bit, chain[1] = combined CRC in; the
// part's end replaces them (parts are chained in stream order on one stream).
// Bit offsets of the blocks (an exclusive sum of their bit lengths from chain[0]) and the
// combined CRC (compress.c:826-828: c = rotl(c, 1) ^ bcrc[b] per block, i.e. rotl(c0, nb) xor
// the xor of rotl(bcrc[b], nb - 1 - b)), one workgroup: a serial walk of ~1100 blocks was
// ~175 us of dependent loads on the critical path.
constexpr uint32_t kOffT = 1024;
__global__ void __launch_bounds__(kOffT) k_offsets(const uint32_t* __restrict__ info, const uint32_t* __restrict__ bcrc,
                                                   uint32_t nb, uint64_t* __restrict__ chain,
                                                   uint64_t* __restrict__ boffbits) {
  __shared__ uint64_t wsum[kOffT / 64];
  __shared__ uint32_t wx[kOffT / 64];
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  const uint32_t per = ceil_div(nb, kOffT), b0 = min(nb, t * per), b1 = min(nb, b0 + per);
  uint64_t mine = 0;
  uint32_t x = 0;
  for (uint32_t b = b0; b < b1; b++) {
    mine += info[(size_t)b * 8 + 3];
    const uint32_t r = (nb - 1 - b) & 31u, c = bcrc[b];
    x ^= r ? (c << r) | (c >> (32 - r)) : c;
  }
  // exclusive sum over the threads (64-bit), xor over the workgroup
  uint64_t incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(incl, o, 64);
    if (lane >= (uint32_t)o) incl += y;
  }
  uint32_t xr = x;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) xr ^= (uint32_t)__shfl_xor((int)xr, o, 64);
  if (lane == 63) wsum[w] = incl;
  if (lane == 0) wx[w] = xr;
  __syncthreads();
  const uint64_t start = chain[0];
  uint64_t pre = start;
  for (uint32_t k = 0; k < w; k++) pre += wsum[k];
  uint64_t pos = pre + incl - mine;
  for (uint32_t b = b0; b < b1; b++) {
    boffbits[b] = pos;
    pos += info[(size_t)b * 8 + 3];
  }
  __syncthreads();  // every thread has read chain[0]
  if (t == kOffT - 1) {
    uint64_t tot = start;
    uint32_t xa = 0;
    for (uint32_t k = 0; k < kOffT / 64; k++) {
      tot += wsum[k];
      xa ^= wx[k];
    }
    const uint32_t c0 = (uint32_t)chain[1], r = nb & 31u;
    chain[0] = tot;
    chain[1] = (r ? (c0 << r) | (c0 >> (32 - r)) : c0) ^ xa;
  }
}

__global__ void k_chain_init(uint64_t* __restrict__ chain, uint64_t start_bit, uint32_t comb) {
  if (threadIdx.x == 0) {
    chain[0] = start_bit;
    chain[1] = comb;
  }
}

// MSB-first bit writer ORing big-endian 32-bit words into a zeroed buffer.
struct BitWriter {
  uint32_t* out;
  uint64_t word;   // index of the word the accumulator starts at
  uint64_t acc;    // bits left-aligned: bit 63 = first bit of `word` (+ already flushed)
  uint32_t nacc;   // valid bits in acc (including the leading alignment bits)
  __device__ BitWriter(uint32_t* o, uint64_t bitpos) : out(o), word(bitpos >> 5), acc(0), nacc((uint32_t)(bitpos & 31)) {}
  __device__ __forceinline__ void put(uint32_t nbits, uint32_t v) {
    // nbits <= 32
    if (nbits == 0) return;
    acc |= ((uint64_t)v << (64 - nbits)) >> nacc;
    nacc += nbits;
    if (nacc >= 32) {
      const uint32_t hi = (uint32_t)(acc >> 32);
      if (hi) atomicOr(&out[word], bswap32(hi));
      ++word;
      acc <<= 32;
      nacc -= 32;
    }
  }
  __device__ __forceinline__ void flush() {
    if (nacc > 0) {
      const uint32_t hi = (uint32_t)(acc >> 32);
      if (hi) atomicOr(&out[word], bswap32(hi));
    }
  }
};
// nbits up to 32 may overflow the accumulator when nacc > 32 after a put; put() keeps
// nacc < 32 on exit, so a put of <= 32 bits never loses bits.


// The step's bit buffer holds either the whole step (default) or a window of it: a smaller
// buffer lets more workgroups share a CU, and a step with more bits (high-entropy input) is
// encoded in several windows, each taking the groups that start inside it.
constexpr uint32_t kPackFull = (kT * kGroupSize * kMaxCodeLen + 31) / 32 + 2;
constexpr uint32_t kPackBitsW = 3328;  // words of the bit buffer: 13 KB, 3 workgroups per CU (the whole step, kPackFull words, gives 2)
constexpr uint32_t kPackOv = (kGroupSize * kMaxCodeLen + 31) / 32 + 1;  // words a group can reach past its window
static_assert(kPackBitsW >= kPackFull || kPackBitsW >= 4 * kPackOv, "bit window too small");
constexpr uint32_t kPackWS = kPackBitsW >= kPackFull ? kPackBitsW * 32 : (kPackBitsW - kPackOv) * 32;  // bits per window

struct PackLds {
  alignas(16) uint16_t chunk[kT * kGroupSize + 8];
  uint32_t bits[kPackBitsW];  // one window of the step's payload
};

__global__ void __launch_bounds__(kT) k_pack(const uint16_t* __restrict__ mtfv, const uint32_t* __restrict__ mtf_off,
                                             const uint32_t* __restrict__ nmtf_g, const uint32_t* __restrict__ inuse,
                                             const uint32_t* __restrict__ bcrc, const uint32_t* __restrict__ origptr,
                                             const uint8_t* __restrict__ lens_g, const uint32_t* __restrict__ codes_g,
                                             const uint8_t* __restrict__ sel_g, const uint8_t* __restrict__ selmtf_g,
                                             const uint16_t* __restrict__ gbits_g, const uint32_t* __restrict__ info_g,
                                             const uint64_t* __restrict__ boffbits, uint32_t* __restrict__ out) {
  __shared__ uint8_t len[kNGroups][kMaxAlpha + 2];
  __shared__ uint32_t code[kNGroups][kMaxAlpha];  // code | length << 24 (one LDS read per symbol)
  __shared__ uint32_t sh[8];
  __shared__ PackLds P;
  // gridDim.x workgroups per block: slice 0 also writes the block header, tables and
  // selectors; slice s packs its share of the payload steps from the bit offset of its first
  // group (p_dat + the bits of the groups before it)
  const uint32_t b = blockIdx.y, slice = blockIdx.x;
  const uint32_t* info = info_g + (size_t)b * 8;
  const int ng = (int)info[0];
  const uint32_t nsel = info[1];
  const int alpha = (int)info[2];
  const uint32_t nmtf = nmtf_g[b];
  const uint16_t* mv = mtfv + mtf_off[b];
  for (int i = threadIdx.x; i < ng * kMaxAlpha; i += kT) {
    len[i / kMaxAlpha][i % kMaxAlpha] = lens_g[(size_t)b * kNGroups * kMaxAlpha + i];
    code[i / kMaxAlpha][i % kMaxAlpha] =
        codes_g[(size_t)b * kNGroups * kMaxAlpha + i] | ((uint32_t)lens_g[(size_t)b * kNGroups * kMaxAlpha + i] << 24);
  }
  __syncthreads();
  const uint64_t p0 = boffbits[b];
  uint32_t used16 = 0;
  for (int i = 0; i < 16; i++) {
    const uint32_t w = inuse[b * 8 + (i >> 1)];
    if ((i & 1) ? (w >> 16) : (w & 0xffffu)) used16++;
  }
  const uint64_t p_sel = p0 + 48 + 32 + 1 + 24 + 16 + 16 * used16 + 3 + 15;
  const uint64_t p_tab = p_sel + info[4];
  const uint64_t p_dat = p_tab + info[5];
  // header, symbol map, nGroups, nSelectors: lane 0
  if (slice == 0 && threadIdx.x == 0) {
    BitWriter w(out, p0);
    w.put(24, 0x314159);
    w.put(24, 0x265359);
    w.put(32, bcrc[b]);
    w.put(1, 0);
    w.put(24, origptr[b]);
    uint32_t top = 0;
    for (int i = 0; i < 16; i++) {
      const uint32_t wd = inuse[b * 8 + (i >> 1)];
      const uint32_t half = (i & 1) ? (wd >> 16) : (wd & 0xffffu);
      top = (top << 1) | (half ? 1u : 0u);
    }
    w.put(16, top);
    for (int i = 0; i < 16; i++) {
      const uint32_t wd = inuse[b * 8 + (i >> 1)];
      const uint32_t half = (i & 1) ? (wd >> 16) : (wd & 0xffffu);
      if (!half) continue;
      uint32_t row = 0;
      for (int j = 0; j < 16; j++) row = (row << 1) | ((half >> j) & 1u);
      w.put(16, row);
    }
    w.put(3, (uint32_t)ng);
    w.put(15, nsel);
    w.flush();
  }
  // code-length tables: lane t writes table t
  if (slice == 0 && threadIdx.x < (unsigned)ng) {
    const int t = threadIdx.x;
    uint64_t pos = p_tab;
    for (int u = 0; u < t; u++) {
      int cur = len[u][0];
      uint32_t bits = 5;
      for (int v = 0; v < alpha; v++) {
        const int l = len[u][v];
        bits += 1 + 2 * (uint32_t)(l > cur ? l - cur : cur - l);
        cur = l;
      }
      pos += bits;
    }
    BitWriter w(out, pos);
    int cur = len[t][0];
    w.put(5, (uint32_t)cur);
    for (int v = 0; v < alpha; v++) {
      const int l = len[t][v];
      while (cur < l) {
        w.put(2, 2);
        cur++;
      }
      while (cur > l) {
        w.put(2, 3);
        cur--;
      }
      w.put(1, 0);
    }
    w.flush();
  }
  // selectors (unary MTF codes): thread-blocked ranges
  const uint8_t* smo = selmtf_g + (size_t)b * kMaxSelectors;
  if (slice == 0) {
    const uint32_t per = ceil_div(nsel, kT);
    const uint32_t lo = min(nsel, threadIdx.x * per), hi = min(nsel, lo + per);
    uint32_t bits = 0;
    for (uint32_t g = lo; g < hi; g++) bits += smo[g] + 1u;
    const uint32_t incl = block_incl_sum(bits, sh, (uint32_t*)nullptr);
    BitWriter w(out, p_sel + incl - bits);
    for (uint32_t g = lo; g < hi; g++) {
      const uint32_t j = smo[g];
      w.put(j + 1, (1u << (j + 1)) - 2u);
    }
    w.flush();
  }
  // payload: kT selector groups per step.  The step's symbols are staged in LDS, every lane
  // encodes its group into an LDS bit buffer at its group's offset, and the buffer goes out as
  // whole words (the two boundary words, shared with the neighbouring steps, by atomicOr).
  {
    const uint8_t* selo = sel_g + (size_t)b * kMaxSelectors;
    const uint16_t* gb = gbits_g + (size_t)b * kMaxSelectors;
    const uint32_t nsteps = ceil_div(nsel, kT), sps = ceil_div(nsteps, gridDim.x);
    const uint32_t s0 = min(nsteps, slice * sps), s1 = min(nsteps, s0 + sps);
    uint64_t pos = p_dat;  // bit position of the step
    {
      uint32_t before = 0;
      for (uint32_t g = threadIdx.x; g < s0 * kT; g += kT) before += gb[g];
      uint32_t tot;
      block_incl_sum(before, sh, &tot);
      pos += tot;
    }
    // a step's symbols are read as 16-byte words (block offsets are multiples of 8 values);
    // the next step's words are loaded into registers while this one is encoded
    uint4 q[kCfVec];
    auto load_step = [&](uint32_t g0) {
      const uint32_t lo = g0 * kGroupSize, hi = min(lo + kT * kGroupSize, nmtf);
#pragma unroll
      for (uint32_t k = 0; k < kCfVec; k++) {
        const uint32_t i = lo + 8 * (threadIdx.x + k * kT);
        q[k] = i < hi ? *reinterpret_cast<const uint4*>(mv + i) : make_uint4(0, 0, 0, 0);
      }
    };
    if (s0 < s1) load_step(s0 * kT);
    for (uint32_t g0 = s0 * kT; g0 < s1 * kT; g0 += kT) {
#pragma unroll
      for (uint32_t k = 0; k < kCfVec; k++) {
        const uint32_t j = 8 * (threadIdx.x + k * kT);
        if (j < kT * kGroupSize) *reinterpret_cast<uint4*>(P.chunk + j) = q[k];
      }
      if (g0 + kT < s1 * kT) load_step(g0 + kT);
      const uint32_t g = g0 + threadIdx.x;
      const uint32_t mybits = g < nsel ? gb[g] : 0u;
      uint32_t stepbits;
      const uint32_t gx = block_incl_sum(mybits, sh, &stepbits) - mybits;
      const uint32_t w0 = (uint32_t)(pos & 31);          // bit offset of the step in its first word
      const uint32_t nwords = (w0 + stepbits + 31) >> 5;  // words the step touches
      const uint32_t nwin = (w0 + stepbits + kPackWS - 1) / kPackWS;
      const uint32_t mywin = (w0 + gx) / kPackWS;
      uint32_t* ow = out + (pos >> 5);
      for (uint32_t r = 0; r < nwin; r++) {
        const uint32_t wbw = r * (kPackWS / 32);  // first word of the window
        const uint32_t nw = min(kPackBitsW, nwords - wbw);
        for (uint32_t i = threadIdx.x; i < nw; i += kT) P.bits[i] = 0;
        __syncthreads();
        if (g < nsel && mywin == r) {
          const int t = selo[g];
          // the group's symbols as 25 LDS pair reads into registers, as in k_cf (k_pack 1.05 ->
          // 0.93 ms per GB of text: profiles/r05_ab_pack_pairs.txt)
          const uint32_t* cw = reinterpret_cast<const uint32_t*>(P.chunk + threadIdx.x * kGroupSize);
          uint32_t sym[kGroupSize / 2];
#pragma unroll
          for (int k = 0; k < (int)kGroupSize / 2; k++) sym[k] = cw[k];
          const uint32_t n = min((uint32_t)kGroupSize, nmtf - g * kGroupSize);
          uint32_t bp = w0 + gx - wbw * 32;         // bit position in P.bits
          uint64_t acc = 0;                         // left-aligned pending bits
          uint32_t na = bp & 31;                    // bits in acc, counted from the word start
          uint32_t wi = bp >> 5;
#pragma unroll
          for (int i = 0; i < (int)kGroupSize; i++) {
            if ((uint32_t)i >= n) break;
            const uint32_t cl = code[t][(sym[i >> 1] >> (16 * (i & 1))) & 0xffffu];
            const uint32_t l = cl >> 24;
            acc |= ((uint64_t)(cl & 0xffffffu) << (64 - l)) >> na;
            na += l;
            if (na >= 32) {
              atomicOr(&P.bits[wi++], (uint32_t)(acc >> 32));
              acc <<= 32;
              na -= 32;
            }
          }
          if (na) atomicOr(&P.bits[wi], (uint32_t)(acc >> 32));
        }
        __syncthreads();
        // words shared with the neighbouring steps, or with the previous / next window, are ORed
        for (uint32_t i = threadIdx.x; i < nw; i += kT) {
          const uint32_t v = bswap32(P.bits[i]);
          const uint32_t gi = wbw + i;
          const bool shared = gi == 0 || gi + 1 == nwords || (r > 0 && i < kPackOv) ||
                              (r + 1 < nwin && i >= kPackWS / 32);
          if (shared) {
            if (v) atomicOr(&ow[gi], v);
          } else {
            ow[gi] = v;
          }
        }
        __syncthreads();
      }
      pos += stepbits;
    }
  }
}

// Stream header ("BZh" + level) and/or trailer (0x177245385090 + combined CRC).
__global__ void k_frame(uint32_t* __restrict__ out, int header, uint64_t hdr_bit, int level, int trailer,
                        const uint64_t* __restrict__ chain) {
  const uint64_t* tpos = chain;
  const uint32_t comb_v = (uint32_t)chain[1];
  const uint32_t* comb = &comb_v;
  if (threadIdx.x != 0) return;
  if (header) {
    BitWriter w(out, hdr_bit);
    w.put(8, 'B');
    w.put(8, 'Z');
    w.put(8, 'h');
    w.put(8, (uint32_t)('0' + level));
    w.flush();
  }
  if (trailer) {
    BitWriter w(out, *tpos);
    w.put(24, 0x177245);
    w.put(24, 0x385090);
    w.put(32, *comb);
    w.flush();
  }
}

}  // namespace

void code_tables(Workspace& ws, const Rle1Result& r, const MtfResult& m, uint32_t nb, CodeTables& t, hipStream_t st,
                 hipStream_t st2) {
  const size_t nbx = std::max<uint32_t>(nb, 1);
  t.lens = ws.u8("code_lens", nbx * kNGroups * kMaxAlpha);
  t.codes = ws.u32("code_codes", nbx * kNGroups * kMaxAlpha);
  t.sel = ws.u8("code_sel", nbx * kMaxSelectors);
  t.selmtf = ws.u8("code_selmtf", nbx * kMaxSelectors);
  t.gbits = ws.u16("code_gbits", nbx * kMaxSelectors);
  t.info = ws.u32("code_info", nbx * 8);
  t.bbits = ws.typed<uint64_t>("code_bbits", nbx + 2);
  uint32_t* rf = ws.u32("code_rf", nbx * kNGroups * kMaxAlpha);
  // k_huff_spec: per-table words (zero between launches: the last workgroup of a table resets
  // its word) and round-2 lengths
  uint32_t* hword = ws.u32z("code_hword", nbx * kNGroups);
  uint8_t* hscratch = ws.u8("code_hscratch", nbx * kNGroups * kMaxAlpha);
  if (nb == 0) return;
  HIP_OK(hipMemsetAsync(t.info, 0, nbx * 8 * 4, st));
  // Blocks are independent, and k_huff is a latency chain with a small grid that leaves the
  // device mostly idle: with a second stream the blocks run as two halves whose k_cf and
  // k_huff launches interleave (one half's selection beside the other half's Huffman).
  const bool split = st2 != nullptr && nb >= 64;
  hipEvent_t e_in = nullptr, e_out = nullptr;
  if (split) {  // (the workspace's events 2 and 3: no event created per call)
    e_in = ws.side_event(2);
    e_out = ws.side_event(3);
    HIP_OK(hipEventRecord(e_in, st));
    HIP_OK(hipStreamWaitEvent(st2, e_in, 0));
  }
  const uint32_t half = split ? nb / 2 : nb;
  for (int h = 0; h < (split ? 2 : 1); h++) {
    const uint32_t b0 = h ? half : 0, n = h ? nb - half : half;
    hipStream_t s = h ? st2 : st;
    const uint32_t nt = n * (uint32_t)kNGroups;
    const bool spec = nt <= huff_spec_max();
    k_init_tables<<<n, 64, 0, s>>>(b0, m.nmtf, m.freq, r.ninuse, t.lens, rf);
    HIP_OK(hipGetLastError());
    for (int it = 0; it < kIters; it++) {
      k_cf<<<dim3(slices_for(n, kCfSlices), n), kT, 0, s>>>(b0, m.mtfv, m.mtf_off, m.nmtf, t.lens, t.sel, rf, t.gbits, t.info, 0);
      HIP_OK(hipGetLastError());
      if (nt >= huff_lanes_min())
        k_huff_lanes<<<ceil_div(nt, (uint32_t)kHuffLanes), 64, 0, s>>>(b0, n, m.nmtf, r.ninuse, rf, t.lens);
      else if (spec)
        k_huff_spec<<<2 * nt, 64, 0, s>>>(b0, nt, m.nmtf, r.ninuse, rf, t.lens, hword, hscratch);
      else
        k_huff<<<nt, 64, 0, s>>>(b0, m.nmtf, r.ninuse, rf, t.lens);
      HIP_OK(hipGetLastError());
    }
    k_cf<<<dim3(slices_for(n, kCfSlices), n), kT, 0, s>>>(b0, m.mtfv, m.mtf_off, m.nmtf, t.lens, t.sel, rf, t.gbits, t.info, 1);
    HIP_OK(hipGetLastError());
    k_final<<<n, kT, 0, s>>>(b0, m.nmtf, r.ninuse, r.inuse, t.lens, t.codes, t.sel, t.selmtf, t.info);
    HIP_OK(hipGetLastError());
  }
  if (split) {
    HIP_OK(hipEventRecord(e_out, st2));
    HIP_OK(hipStreamWaitEvent(st, e_out, 0));
  }
}

uint64_t code_emit(Workspace& ws, const std::vector<CodePart>& parts, int level, bool final_batch, StreamCarry& carry,
                   uint8_t* out, uint64_t out_cap, hipStream_t st) {
  uint64_t* chain = ws.typed<uint64_t>("code_chain", 4);
  const bool header = !carry.header_done;
  const uint64_t start_bit = carry.carry_bits + (header ? 32 : 0);
  k_chain_init<<<1, 64, 0, st>>>(chain, start_bit, carry.combined_crc);
  HIP_OK(hipGetLastError());
  for (const CodePart& p : parts) {
    if (p.nb == 0) continue;
    k_offsets<<<1, kOffT, 0, st>>>(p.t->info, p.r->bcrc, p.nb, chain, p.t->bbits);
    HIP_OK(hipGetLastError());
  }
  uint64_t hch[2];
  ws.read_small(hch, chain, 16, st);
  const uint64_t total_bits = hch[0];
  const uint32_t comb_h = (uint32_t)hch[1];
  const uint64_t end_bits = total_bits + (final_batch ? 80 : 0);
  const uint64_t need = ceil_div64(end_bits, 32) * 4 + 8;
  if (need > out_cap) throw OutBuffFull{};
  HIP_OK(hipMemsetAsync(out, 0, need, st));
  if (carry.carry_bits) HIP_OK(hipMemcpyAsync(out, &carry.carry_byte, 1, hipMemcpyHostToDevice, st));
  for (const CodePart& p : parts) {
    if (p.nb == 0) continue;
    const CodeTables& t = *p.t;
    k_pack<<<dim3(slices_for(p.nb, kPackSlices), p.nb), kT, 0, st>>>(p.m->mtfv, p.m->mtf_off, p.m->nmtf, p.r->inuse, p.r->bcrc, p.origptr,
                                                 t.lens, t.codes, t.sel, t.selmtf, t.gbits, t.info, t.bbits,
                                                 (uint32_t*)out);
    HIP_OK(hipGetLastError());
  }
  if (header || final_batch) {
    k_frame<<<1, 64, 0, st>>>((uint32_t*)out, header ? 1 : 0, carry.carry_bits, level, final_batch ? 1 : 0, chain);
    HIP_OK(hipGetLastError());
  }
  carry.header_done = true;
  carry.combined_crc = comb_h;
  if (final_batch) {
    carry.carry_bits = 0;
    carry.carry_byte = 0;
    return ceil_div64(end_bits, 8);
  }
  const uint64_t full = end_bits >> 3;
  carry.carry_bits = (uint8_t)(end_bits & 7);
  if (carry.carry_bits) {
    HIP_OK(hipMemcpyAsync(&carry.carry_byte, out + full, 1, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  } else {
    carry.carry_byte = 0;
  }
  return full;
}

uint64_t code_stage(Workspace& ws, const Rle1Result& r, const MtfResult& m, const uint32_t* origptr, uint32_t nb,
                    int level, bool final_batch, StreamCarry& carry, uint8_t* out, uint64_t out_cap, hipStream_t st) {
  CodeTables t;
  code_tables(ws, r, m, nb, t, st);
  std::vector<CodePart> parts{CodePart{&r, &m, &t, origptr, nb}};
  return code_emit(ws, parts, level, final_batch, carry, out, out_cap, st);
}

void code_lengths_test(Workspace& ws, const uint32_t* d_freq, const int32_t* d_alpha, uint32_t n, int max_len,
                       uint8_t* d_lens, hipStream_t st) {
  if (n == 0) return;
  uint32_t* word = ws.u32z("test_hword", n);
  uint8_t* scratch = ws.u8("test_hscratch", (size_t)n * kMaxAlpha);
  if (huff_lanes_min() == 0) {  // BZG_HUFF_LANES_MIN=0: the lane-per-table routine (its parity tests)
    k_code_lengths_lanes<<<ceil_div(n, (uint32_t)kHuffLanes), 64, 0, st>>>(d_freq, d_alpha, n, max_len, d_lens);
  } else if (n <= huff_spec_max()) {
    k_code_lengths_spec<<<2 * n, 64, 0, st>>>(d_freq, d_alpha, n, max_len, d_lens, word, scratch);
  } else {
    k_code_lengths_test<<<n, 64, 0, st>>>(d_freq, d_alpha, max_len, d_lens);
  }
  HIP_OK(hipGetLastError());
}

}  // namespace bzg
