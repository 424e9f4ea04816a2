// decomp.hip -- block-parallel .bz2 decompression on the GPU.
//
// The reference decodes a stream bit-serially, one block after another (decompress.c:232-…,
// the decode tables of huffman.c:180-236, the inverse BWT and un-RLE1 of bzlib.c:531-677).
// Here every block is decoded at once:
//   0. block boundaries: every block-header / end-of-stream magic of the stream, at any bit
//      offset (magic.hip).  A magic can also occur by chance inside coded data, so each
//      candidate is decoded speculatively and the real blocks are the chain that starts at
//      bit 32 and continues at each block's end bit.
//   1. k_dec_huff, one wave per candidate: header, selectors (unary + MTF), delta-coded code
//      lengths, canonical decode tables (9-bit lookup table + per-length limits in LDS), then
//      the symbol loop -- Huffman decode, RUNA/RUNB run lengths, inverse MTF -- writing the
//      block's BWT last column L.  All decoder state is wave-uniform; the 64 lanes hold the
//      bit window (64 words + 64 prefetched) and the MTF list (4 entries per lane, a move to
//      front is one lane shift), and stage output bytes in LDS for 256-byte stores.
//   2. k_dec_tt, a workgroup per block: stable counting sort of L (per-wave byte histograms
//      from 8-ballot byte matching), giving for every row j of the sorted rotations the
//      packed successor Q[j] = (i << 8) | L[i] with LF(i) = j.
//   3. k_dec_walk, a workgroup per block: the text is the walk j <- Q[j] >> 8 from origPtr,
//      emitting Q[j] & 0xff (bzlib_private.h BZ_GET_FAST).  The walk is split at every 256th
//      row (a ruling set): each thread walks its splitters' segments to the next splitter,
//      one thread chains the segments (LDS) into output offsets, and the segments are walked
//      again writing bytes.  A walk that closes its cycle before n steps (periodic blocks)
//      repeats with the cycle's period, as the reference's n-step walk does.
//   4. un-RLE1 as a 5-state machine (state = length of the current run since the last count
//      byte, 4 = the next byte is a count).  k_dec_rle_scan composes each chunk's transition
//      function for all 5 start states and chains the chunks; k_dec_rle_emit replays each
//      chunk from its start state into the output with its CRC piece, and the block CRC is
//      the GF(2) fold of the pieces.
// The host checks the block CRCs and the combined CRC (bzlib.c BZ2_bzDecompress) and maps the
// outcome to the return codes BZ2_bzBuffToBuffDecompress gives (bzlib.c:1361-1410): an error
// in block k is reported after blocks < k are output; output that does not fit is
// BZ_OUTBUFF_FULL; a stream that ends early is BZ_UNEXPECTED_EOF.
#include <algorithm>
#include <vector>

#include "stages.h"

#define BZ_OK 0
#define BZ_DATA_ERROR (-4)
#define BZ_DATA_ERROR_MAGIC (-5)
#define BZ_UNEXPECTED_EOF (-7)
#define BZ_OUTBUFF_FULL (-8)

namespace bzg {
namespace {

constexpr int kLutBits = 10;
constexpr int kMaxDecLen = 20;          // BZ_MAX_DECODE_LEN (bzlib_private.h:141)
constexpr uint32_t kSelCap = 18002;     // BZ_MAX_SELECTORS: more is a data error (decompress.c:380)
constexpr uint32_t kSplit = 256;        // ruling-set spacing of the inverse-BWT walk
constexpr uint32_t kMaxSplit = 900000 / kSplit + 2;
constexpr uint32_t kRleChunks = 256;    // un-RLE1 chunks (threads) per block
constexpr uint32_t kBatch = 4096;       // block candidates decoded per pass

constexpr uint32_t kMtfChunk = 1024;    // symbols per inverse-MTF chunk
constexpr int kStatusCap = -100;        // more symbols than a block can hold (a data error)

struct DecRes {
  int32_t status;   // phase 1: 0 (EOB reached), BZ_DATA_ERROR, BZ_UNEXPECTED_EOF or kStatusCap
  uint32_t nsym;    // symbols before EOB (or before the failure)
  uint64_t end_bit; // first bit after the block
  uint32_t origptr;
  uint32_t crc;     // stored block CRC
  uint32_t rand;    // randomised-block bit
  uint32_t ninuse;
  uint32_t nblock;  // phase 2: bytes of L
  uint32_t err2;    // phase 2: index of the first symbol the reference rejects (~0: none)
};

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, uint32_t l) {
  return ((uint64_t)rdlane((uint32_t)(v >> 32), l) << 32) | rdlane((uint32_t)v, l);
}

// Big-endian 32-bit word w of the stream (bytes past the end read as zero).
__device__ __forceinline__ uint32_t stream_word(const uint8_t* __restrict__ in, uint64_t nbytes, uint64_t w) {
  const uint64_t b = 4 * w;
  if (b + 4 <= nbytes) return ((uint32_t)in[b] << 24) | ((uint32_t)in[b + 1] << 16) | ((uint32_t)in[b + 2] << 8) | in[b + 3];
  uint32_t v = 0;
  for (int k = 0; k < 4; k++) v = (v << 8) | (b + k < nbytes ? (uint32_t)in[b + k] : 0u);
  return v;
}

// The same word as stored (little-endian load of the big-endian stream word; bswap32 at use).
__device__ __forceinline__ uint32_t stream_word_raw(const uint8_t* __restrict__ in, uint64_t nbytes, uint64_t w) {
  const uint64_t b = 4 * w;
  if (b + 4 <= nbytes && ((reinterpret_cast<uintptr_t>(in) & 3) == 0)) return reinterpret_cast<const uint32_t*>(in)[w];
  return bswap32(stream_word(in, nbytes, w));
}

// Wave-wide bit window: lane l holds word wbase + l in `cur` and wbase + 64 + l in `nxt`.
// Positions only move forward; peek32 returns the 32 bits starting at absolute bit p.
struct BitWindow {
  const uint8_t* in;
  uint64_t nbytes;
  uint64_t wbase;
  uint32_t cur, nxt;
  __device__ void init(const uint8_t* i, uint64_t nb, uint64_t p) {
    in = i;
    nbytes = nb;
    wbase = p >> 5;
    cur = stream_word(in, nbytes, wbase + __lane_id());
    nxt = stream_word(in, nbytes, wbase + 64 + __lane_id());
  }
  __device__ __forceinline__ uint32_t peek32(uint64_t p) {
    uint64_t off = p - 32 * wbase;
    while (off >= 2048) {
      cur = nxt;
      wbase += 64;
      nxt = stream_word(in, nbytes, wbase + 64 + __lane_id());
      off -= 2048;
    }
    const uint32_t wi = (uint32_t)(off >> 5), sh = (uint32_t)(off & 31);
    const uint32_t hi = rdlane(cur, wi);
    const uint32_t lo = wi < 63 ? rdlane(cur, wi + 1) : rdlane(nxt, 0);
    return sh ? (hi << sh) | (lo >> (32 - sh)) : hi;
  }
  __device__ __forceinline__ uint32_t get(uint64_t& p, uint32_t k) {  // 1 <= k <= 32
    const uint32_t v = peek32(p);
    p += k;
    return k == 32 ? v : v >> (32 - k);
  }
};

// Phase 1, one wave per candidate: header, selectors, code lengths, decode tables, then the
// Huffman symbols of the block (RUNA 0, RUNB 1, MTF value + 1 for 2..nInUse; EOB not stored),
// 64 per vector store.  The symbol loop keeps its whole state in scalar registers: a 64-bit
// bit buffer refilled from the lane-held window, one LDS lookup (10-bit table) per symbol.
__global__ void __launch_bounds__(64) k_dec_huff(const uint8_t* __restrict__ in, uint64_t nbytes,
                                                 const uint64_t* __restrict__ cbit, uint32_t nc, uint32_t nbmax,
                                                 uint32_t symstride, uint16_t* __restrict__ symbuf,
                                                 uint8_t* __restrict__ seqbuf, uint8_t* __restrict__ selbuf,
                                                 DecRes* __restrict__ res, uint64_t* __restrict__ dbg) {
  const uint64_t t_start = clock64();
  uint64_t t_sym = 0;
  // per 10-bit window: total | n << 5 | sym0 << 7 | sym1 << 16 | len0 << 25 -- n = 1 or 2 symbols
  // decoded from the window (a second one only if both fit and the first is not EOB), n = 0:
  // the first code is longer than the window
  __shared__ uint32_t lut[kNGroups * (1u << kLutBits)];
  __shared__ uint16_t perm[kNGroups][kMaxAlpha];         // symbols in canonical order
  __shared__ int32_t limit[kNGroups][kMaxDecLen + 1];
  __shared__ int32_t cbase[kNGroups][kMaxDecLen + 1];
  __shared__ uint8_t lens[kNGroups][kMaxAlpha];
  __shared__ uint32_t cnt[kMaxDecLen + 1];
  __shared__ uint8_t seq[256];
  // windowed chain decoding of the selectors and the symbols (below): stream words in an LDS
  // ring, a window of kWin bit positions decoded at every position, pointer-jump tables
  constexpr uint32_t kWin = 256, kPerLane = kWin / 64, kRing = 256;
  __shared__ uint32_t ring[kRing];         // stream words [rfill - kRing, rfill) at [w % kRing]
  __shared__ uint16_t J[6][kWin + 1];      // J[b][q]: the start 2^b codes after q (kWin: outside)
  __shared__ uint16_t nxa[kWin];           // q + length of the code at q (unclamped)
  __shared__ uint16_t sq[kWin];            // symbol of the code at q (selectors: leading ones)
  const uint32_t c = blockIdx.x;
  if (c >= nc) return;
  const uint32_t lane = __lane_id();
  const uint64_t nbits = 8 * nbytes;
  uint64_t p = cbit[c];
  int status = 0;
  uint32_t origptr = 0, bcrc = 0, rnd = 0, ns = 0;
  BitWindow W;
  W.init(in, nbytes, p);
  uint32_t ninuse = 0, g = 0, nsel = 0, alpha = 0;
  uint64_t rfill = 0;  // the ring holds stream words [rfill - kRing, rfill); the next 128 are in pre0 / pre1
  uint32_t pre0 = 0, pre1 = 0;
  auto ring_init = [&](uint64_t bit) {
    rfill = bit >> 5;
#pragma unroll
    for (uint32_t k = 0; k < kRing / 64; k++)
      ring[(rfill + 64 * k + lane) % kRing] = bswap32(stream_word_raw(in, nbytes, rfill + 64 * k + lane));
    rfill += kRing;
    pre0 = stream_word_raw(in, nbytes, rfill + lane);
    pre1 = stream_word_raw(in, nbytes, rfill + 64 + lane);
    if (lane < 6) J[lane][kWin] = (uint16_t)kWin;
    __builtin_amdgcn_wave_barrier();
  };
  // bits up to `bit` (exclusive) readable from the ring; the window start must stay within the
  // ring's last kRing - 128 words (windows are kWin + 32 bits, far below)
  auto ring_ensure = [&](uint64_t bit) {
    while (((bit + 31) >> 5) >= rfill) {
      ring[(rfill + lane) % kRing] = bswap32(pre0);
      ring[(rfill + 64 + lane) % kRing] = bswap32(pre1);
      rfill += 128;
      pre0 = stream_word_raw(in, nbytes, rfill + lane);
      pre1 = stream_word_raw(in, nbytes, rfill + 64 + lane);
    }
    __builtin_amdgcn_wave_barrier();
  };
  auto ring_peek = [&](uint64_t x) -> uint32_t {  // the 32 bits at absolute bit x (ensured)
    const uint32_t w = (uint32_t)(x >> 5), sh = (uint32_t)(x & 31);
    const uint32_t hi = ring[w % kRing], lo = ring[(w + 1) % kRing];
    return sh ? (hi << sh) | (lo >> (32 - sh)) : hi;
  };
  // the chain 0 -> J[0][0] -> ... through the window: J[1..5] by pointer jumping, then lane i
  // composes its i steps; jq holds J[0] of this lane's positions on entry.  Returns s_lane.
  auto chain_starts = [&](uint32_t (&jq)[kPerLane]) -> uint32_t {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t b = 1; b < 6; b++) {
#pragma unroll
      for (uint32_t k = 0; k < kPerLane; k++) jq[k] = J[b - 1][jq[k]];
#pragma unroll
      for (uint32_t k = 0; k < kPerLane; k++) J[b][lane + 64 * k] = (uint16_t)jq[k];
      __builtin_amdgcn_wave_barrier();
    }
    uint32_t s = 0;
#pragma unroll
    for (uint32_t b = 0; b < 6; b++)
      if ((lane >> b) & 1u) s = J[b][s];
    return s;
  };

  // ---- block header (decompress.c:306-352): magic (found by the scan), CRC, rand bit, origPtr
  // the reference checks origPtr before it reads the 16 mapping bits (decompress.c:348-351)
  if (p + 48 + 32 + 1 + 24 > nbits) { status = BZ_UNEXPECTED_EOF; goto done; }
  p += 48;
  bcrc = W.get(p, 32);
  rnd = W.get(p, 1);
  origptr = W.get(p, 24);
  if (origptr > nbmax) { status = BZ_DATA_ERROR; goto done; }
  if (p + 16 > nbits) { status = BZ_UNEXPECTED_EOF; goto done; }
  // ---- symbol map (decompress.c:354-370)
  {
    const uint32_t used16 = W.get(p, 16);
    for (uint32_t j = 0; j < 16; j++) {
      if (!((used16 >> (15 - j)) & 1u)) continue;
      if (p + 16 > nbits) { status = BZ_UNEXPECTED_EOF; goto done; }
      const uint32_t w = W.get(p, 16);
      for (uint32_t i = 0; i < 16; i++)
        if ((w >> (15 - i)) & 1u) {
          if (lane == 0) seq[ninuse] = (uint8_t)(16 * j + i);
          ninuse++;
        }
    }
  }
  if (ninuse == 0) { status = BZ_DATA_ERROR; goto done; }
  alpha = ninuse + 2;
  // ---- selectors (decompress.c:375-410): unary MTF indices, then their inverse MTF
  if (p + 18 > nbits) { status = BZ_UNEXPECTED_EOF; goto done; }
  g = W.get(p, 3);
  nsel = W.get(p, 15);
  if (g < 2 || g > 6 || nsel < 1 || nsel > kSelCap) { status = BZ_DATA_ERROR; goto done; }
  // The unary codes are decoded as chains through windows of kWin bit positions (the leading
  // 1 bits at every position at once, as for the symbols below), the MTF of the table numbers
  // then runs over the window's codes in order (a serial loop per selector was most of the
  // header's time: ~12,000 selectors per text block).
  ring_init(p);
  {
    uint32_t pos = 0x543210u;  // MTF list of table numbers, 4 bits per entry
    uint8_t* sdst = selbuf + (size_t)c * kSelCap;
    uint64_t a = p;
    uint32_t i0 = 0;
    while (i0 < nsel) {
      ring_ensure(a + kWin + 32);
      uint32_t jq[kPerLane];
#pragma unroll
      for (uint32_t k = 0; k < kPerLane; k++) {
        const uint32_t q = lane + 64 * k;
        const uint32_t v = ring_peek(a + q);
        const uint32_t o = (~v == 0u) ? 32u : (uint32_t)__builtin_clz(~v);  // leading 1 bits
        sq[q] = (uint16_t)o;
        jq[k] = o >= g ? kWin : min(q + o + 1, kWin);  // (the g-th 1 bit is an error: the chain stops)
        J[0][q] = (uint16_t)jq[k];
      }
      const uint32_t s = chain_starts(jq);
      const bool in_win = i0 + lane < nsel && s < kWin;
      const uint32_t m = (uint32_t)__popcll(__ballot(in_win));
      const uint32_t o = in_win ? sq[s] : 0u;
      const uint64_t at = a + s;
      const uint32_t need = o >= g ? g : o + 1;
      const uint64_t eofm = __ballot(in_win && at + need > nbits), errm = __ballot(in_win && o >= g);
      const uint32_t ieof = eofm ? (uint32_t)__builtin_ctzll(eofm) : 64u;
      const uint32_t ierr = errm ? (uint32_t)__builtin_ctzll(errm) : 64u;
      const uint32_t cnt = min(m, min(ieof, ierr));
      uint32_t selv = 0;
      for (uint32_t j = 0; j < cnt; j++) {
        const uint32_t oj = rdlane(o, j);
        const uint32_t t = (pos >> (4 * oj)) & 0xfu;
        if (oj) {
          const uint32_t low = pos & ((1u << (4 * oj)) - 1u);
          pos = (pos & ~((1u << (4 * (oj + 1))) - 1u)) | (low << 4) | t;
        }
        selv = lane == j ? t : selv;
      }
      if (lane < cnt) sdst[i0 + lane] = (uint8_t)selv;
      if (cnt < m) {  // at code cnt: the stream ends (checked first), or its g-th 1 bit
        p = rdlane64(at, cnt);
        status = ieof <= ierr ? BZ_UNEXPECTED_EOF : BZ_DATA_ERROR;
        goto done;
      }
      a = rdlane64(at + o + 1, m - 1);
      i0 += m;
    }
    p = a;
  }
  // ---- code lengths (decompress.c:412-425): 5-bit start, then per symbol 0 | 1(0:+1, 1:-1)
  for (uint32_t t = 0; t < g; t++) {
    if (p + 5 > nbits) { status = BZ_UNEXPECTED_EOF; goto done; }
    ring_ensure(p + 32);
    uint32_t curr = ring_peek(p) >> 27;
    p += 5;
    for (uint32_t s = 0; s < alpha; s++) {
      for (;;) {
        if (curr < 1 || curr > (uint32_t)kMaxDecLen) { status = BZ_DATA_ERROR; goto done; }
        if (p + 2 > nbits) { status = BZ_UNEXPECTED_EOF; goto done; }
        ring_ensure(p + 32);
        const uint32_t two = ring_peek(p) >> 30;
        if (!(two & 2u)) {
          p += 1;
          break;
        }
        p += 2;
        curr = (two & 1u) ? curr - 1 : curr + 1;
      }
      if (lane == 0) lens[t][s] = (uint8_t)curr;
    }
  }
  __syncthreads();
  // ---- decode tables (huffman.c:180-236 accepts exactly the complete codes: Kraft sum 1)
  for (uint32_t t = 0; t < g; t++) {
    if (lane <= (uint32_t)kMaxDecLen) cnt[lane] = 0;
    __syncthreads();
    for (uint32_t s = lane; s < alpha; s += 64) atomicAdd(&cnt[lens[t][s]], 1u);
    __syncthreads();
    uint32_t kraft = 0;
    for (int l = 1; l <= kMaxDecLen; l++) kraft += cnt[l] << (kMaxDecLen - l);
    kraft = uni(kraft);
    if (kraft != (1u << kMaxDecLen)) { status = BZ_DATA_ERROR; goto done; }
    if (lane == 0) {
      int32_t code = 0, off = 0;
      for (int l = 1; l <= kMaxDecLen; l++) {
        const int32_t k = (int32_t)cnt[l];
        limit[t][l] = code + k - 1;
        cbase[t][l] = off - code;
        cnt[l] = (uint32_t)off;  // becomes the running slot of length l
        off += k;
        code = (code + k) << 1;
      }
      for (uint32_t s = 0; s < alpha; s++) perm[t][cnt[lens[t][s]]++] = (uint16_t)s;
    }
    __syncthreads();
    for (uint32_t x = lane; x < (1u << kLutBits); x += 64) {
      uint32_t e = 0;
      for (int l = 1; l <= kLutBits; l++) {
        const int32_t v = (int32_t)(x >> (kLutBits - l));
        if (v <= limit[t][l]) {
          const uint32_t s0 = perm[t][cbase[t][l] + v];
          e = (uint32_t)l | (1u << 5) | (s0 << 7) | ((uint32_t)l << 25);
          if (s0 != ninuse + 1) {  // a second code inside the window
            const uint32_t x2 = (x << l) & ((1u << kLutBits) - 1);
            for (int l1 = 1; l1 <= kLutBits - l; l1++) {
              const int32_t v1 = (int32_t)(x2 >> (kLutBits - l1));
              if (v1 <= limit[t][l1]) {
                const uint32_t s1 = perm[t][cbase[t][l1] + v1];
                e = (uint32_t)(l + l1) | (2u << 5) | (s0 << 7) | (s1 << 16) | ((uint32_t)l << 25);
                break;
              }
            }
          }
          break;
        }
      }
      lut[t * (1u << kLutBits) + x] = e;
    }
    __syncthreads();
  }
  // ---- symbols (decompress.c:444-664, the Huffman half; MTF and runs are phase 2)
  // Group-parallel decoding.  The 50 symbols of a selector group share one table, so a window
  // of kWin bit positions from the group's first symbol is decoded at EVERY position at once
  // (64 lanes x 4: the length and symbol of the code that would start there), and the chain of
  // real symbol starts 0 -> next(0) -> next(next(0)) ... is read off by pointer jumping (5
  // rounds to build next^2 .. next^32, then 6 rounds in which lane i composes its i steps),
  // instead of 50 dependent table lookups on one lane (that serial loop was 114 ms of a 166 ms
  // decode of 1 GB of text: one wave per block, ~700 cycles per lookup).  A group whose codes
  // run past the window continues in the next window.  Every symbol (EOB and run digits
  // included) takes the next slot of its group; a symbol past the last selector's group is a
  // data error (decompress.c GET_MTF_VAL), a code running past the stream end an unexpected EOF.
  {
    const uint32_t eob = ninuse + 1;
    const uint8_t* ssrc = selbuf + (size_t)c * kSelCap;
    uint16_t* sdst = symbuf + (size_t)c * symstride;
    // the serial decoder's cap (more symbols than a block can hold): stop at the first multiple
    // of 64 above nbmax
    const uint32_t cap = 64u * (nbmax / 64u + 1u);
    t_sym = clock64();
    uint64_t a = p;  // absolute bit of the next code
    uint32_t gi = 0, sreg = 0;
    bool stop = false;
    while (!stop) {
      if (gi == nsel) { status = BZ_DATA_ERROR; break; }
      if ((gi & 63) == 0) sreg = gi + lane < nsel ? ssrc[gi + lane] : 0u;  // 64 selectors at a time
      const uint32_t tb = uni(rdlane(sreg, gi & 63)) << kLutBits;
      const uint32_t t = tb >> kLutBits;
      gi++;
      uint32_t need = kGroupSize;
      while (need > 0) {
        ring_ensure(a + kWin + 32);
        // the code at every position of the window
        uint32_t jq[kPerLane];
#pragma unroll
        for (uint32_t k = 0; k < kPerLane; k++) {
          const uint32_t q = lane + 64 * k;
          const uint32_t v = ring_peek(a + q);
          const uint32_t e = lut[tb + (v >> (32 - kLutBits))];
          uint32_t len, s0;
          if ((e & 0x60u) == 0) {  // longer than the table: canonical limits per length
            len = kLutBits + 1;
            for (int l = kLutBits + 1; l < kMaxDecLen; l++) len += (int32_t)(v >> (32 - l)) > limit[t][l] ? 1u : 0u;
            s0 = perm[t][cbase[t][len] + (int32_t)(v >> (32 - len))];
          } else {
            len = e >> 25;
            s0 = (e >> 7) & 511u;
          }
          nxa[q] = (uint16_t)(q + len);
          sq[q] = (uint16_t)s0;
          jq[k] = min(q + len, kWin);
          J[0][q] = (uint16_t)jq[k];
        }
        const uint32_t s = chain_starts(jq);
        const bool in_win = lane < need && s < kWin;
        const uint32_t m = (uint32_t)__popcll(__ballot(in_win));  // codes of the group in this window
        const uint32_t sym = in_win ? sq[s] : 0u;
        const uint64_t endb = in_win ? a + nxa[s] : 0ull;
        const uint64_t eofm = __ballot(in_win && endb > nbits), eobm = __ballot(in_win && sym == eob);
        const uint32_t ieof = eofm ? (uint32_t)__builtin_ctzll(eofm) : 64u;
        const uint32_t ieob = eobm ? (uint32_t)__builtin_ctzll(eobm) : 64u;
        uint32_t cnt = min(m, min(ieof, ieob));  // codes emitted (an EOF code or EOB is not)
        const bool capped = ns + cnt >= cap;
        if (capped) cnt = cap - ns;
        if (lane < cnt) sdst[ns + lane] = (uint16_t)sym;
        ns += cnt;
        if (capped) {
          status = kStatusCap;
          a = rdlane64(endb, cnt - 1);
          stop = true;
          break;
        }
        if (ieof < m && ieof <= ieob) {  // the stream ends inside this code
          status = BZ_UNEXPECTED_EOF;
          a = ieof ? rdlane64(endb, ieof - 1) : a;
          stop = true;
          break;
        }
        if (ieob < m) {  // end of block
          a = rdlane64(endb, ieob);
          stop = true;
          break;
        }
        a = rdlane64(endb, m - 1);
        need -= m;
      }
    }
    p = a;
  }
done:
  if (lane < 64) reinterpret_cast<uint32_t*>(seqbuf + (size_t)c * 256)[lane] = reinterpret_cast<const uint32_t*>(seq)[lane];
  if (dbg && lane == 0) {
    const uint64_t t_end = clock64();
    dbg[4 * c] = t_sym ? t_sym - t_start : 0;
    dbg[4 * c + 1] = t_sym ? t_end - t_sym : 0;
    dbg[4 * c + 2] = ns;
    dbg[4 * c + 3] = p - cbit[c];
  }
  if (lane == 0) {
    DecRes r;
    r.status = status;
    r.nsym = ns;
    r.end_bit = p;
    r.origptr = origptr;
    r.crc = bcrc;
    r.rand = rnd;
    r.ninuse = ninuse;
    r.nblock = 0;
    r.err2 = ~0u;
    res[c] = r;
  }
}

// Phase 2a, one lane per chunk of kMtfChunk symbols: inverse MTF from a symbolic initial list
// (position k holds token k, "entry k of the chunk's real initial list").  Writes a token per
// symbol (a run digit gets the front token) and the chunk's final list of tokens.  The list
// is 64 words per lane in LDS ([word][lane]: conflict-free); word 0 stays in a register.
__global__ void __launch_bounds__(64) k_dec_mtf_sym(const uint16_t* __restrict__ symbuf, uint32_t symstride,
                                                    const uint32_t* __restrict__ chunk_cand,
                                                    const uint32_t* __restrict__ chunk_j, uint32_t nchunks,
                                                    const DecRes* __restrict__ res, uint8_t* __restrict__ tokbuf,
                                                    uint32_t* __restrict__ permbuf) {
  __shared__ uint32_t Lw[64][64];
  const uint32_t lane = threadIdx.x;
  const uint32_t q = blockIdx.x * 64 + lane;
  if (q >= nchunks) return;
  const uint32_t c = chunk_cand[q];
  const uint32_t lo = chunk_j[q] * kMtfChunk, hi = min(res[c].nsym, lo + kMtfChunk);
  for (uint32_t w = 1; w < 64; w++) Lw[w][lane] = (4 * w) | ((4 * w + 1) << 8) | ((4 * w + 2) << 16) | ((4 * w + 3) << 24);
  uint32_t w0 = 0x03020100u;
  const uint16_t* S = symbuf + (size_t)c * symstride;
  uint8_t* T = tokbuf + (size_t)c * symstride;
  for (uint32_t i = lo; i < hi; i += 4) {
    const uint2 q4 = *reinterpret_cast<const uint2*>(S + i);
    const uint32_t sv[4] = {q4.x & 0xffffu, q4.x >> 16, q4.y & 0xffffu, q4.y >> 16};
    uint32_t tok4 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (i + k >= hi) break;
      const uint32_t s = sv[k];
      uint32_t v;
      if (s <= 1) {
        v = w0 & 0xffu;
      } else {
        const uint32_t r = s - 1;
        if (r < 4) {
          v = (w0 >> (8 * r)) & 0xffu;
          const uint32_t m = r == 3 ? 0xffffffffu : ((1u << (8 * (r + 1))) - 1u);
          w0 = (((w0 << 8) | v) & m) | (w0 & ~m);
        } else {
          const uint32_t wr = r >> 2, br = r & 3u;
          const uint32_t x = Lw[wr][lane];
          v = (x >> (8 * br)) & 0xffu;
          uint32_t carry = w0 >> 24;
          w0 = (w0 << 8) | v;
          for (uint32_t k2 = 1; k2 < wr; k2++) {
            const uint32_t y = Lw[k2][lane];
            Lw[k2][lane] = (y << 8) | carry;
            carry = y >> 24;
          }
          const uint32_t m = br == 3 ? 0xffffffffu : ((1u << (8 * (br + 1))) - 1u);
          Lw[wr][lane] = (((x << 8) | carry) & m) | (x & ~m);
        }
      }
      tok4 |= v << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(T + i) = tok4;
  }
  uint32_t* P = permbuf + (size_t)q * 64;
  P[0] = w0;
  for (uint32_t w = 1; w < 64; w++) P[w] = Lw[w][lane];
}

// Phase 2b, a workgroup per block: the real initial list of every chunk,
// init[j + 1][k] = init[j][perm_j[k]], from the block's in-use bytes ascending.
__global__ void __launch_bounds__(256) k_dec_mtf_chain(const uint32_t* __restrict__ slot,
                                                       const uint32_t* __restrict__ chunk_first,
                                                       const DecRes* __restrict__ res, const uint8_t* __restrict__ seqbuf,
                                                       const uint32_t* __restrict__ permbuf, uint8_t* __restrict__ initbuf) {
  __shared__ uint8_t sh[256];
  const uint32_t b = blockIdx.x, c = slot[b], k = threadIdx.x;
  const uint32_t q0 = chunk_first[b], nch = chunk_first[b + 1] - q0;
  uint32_t cur = seqbuf[(size_t)c * 256 + k];
  const uint8_t* P = reinterpret_cast<const uint8_t*>(permbuf);
  for (uint32_t j = 0; j < nch; j++) {
    initbuf[(size_t)(q0 + j) * 256 + k] = (uint8_t)cur;
    sh[k] = (uint8_t)cur;
    __syncthreads();
    const uint32_t pk = P[(size_t)(q0 + j) * 256 + k];
    cur = sh[pk];
    __syncthreads();
  }
}

// Phase 2c, a workgroup per block: run lengths (RUNA/RUNB digits, bijective base 2), output
// positions by a block-wide scan, the reference's limits (a run that passes 2^20 before its
// next digit, more than nblockMAX bytes: decompress.c:486-500, 520-525) as the index of the
// first failing symbol, and the BWT column L written as 4-byte words.
__global__ void __launch_bounds__(1024) k_dec_expand(const uint32_t* __restrict__ slot,
                                                     const uint32_t* __restrict__ chunk_first, uint32_t nbmax,
                                                     uint32_t symstride, const uint16_t* __restrict__ symbuf,
                                                     const uint8_t* __restrict__ tokbuf,
                                                     const uint8_t* __restrict__ initbuf, DecRes* __restrict__ res,
                                                     uint8_t* __restrict__ lbuf) {
  __shared__ uint32_t spos[1024];   // output position of each symbol of the tile, relative to the tile
  __shared__ uint8_t sbyte[1024];
  __shared__ uint64_t sh64[16];
  __shared__ int32_t shi[16];
  __shared__ uint32_t err_sh;
  __shared__ uint64_t carry_rsp_sh;
  const uint32_t b = blockIdx.x, c = slot[b], tid = threadIdx.x;
  const uint32_t ns = res[c].nsym;
  const bool eob_reached = res[c].status == 0;
  const uint16_t* S = symbuf + (size_t)c * symstride;
  const uint8_t* T = tokbuf + (size_t)c * symstride;
  const uint8_t* I = initbuf + (size_t)chunk_first[b] * 256;
  uint8_t* L = lbuf + (size_t)c * nbmax;
  if (tid == 0) {
    err_sh = ~0u;
    carry_rsp_sh = 0;
  }
  uint64_t carry_pos = 0;
  int32_t carry_lnd = -1;
  __syncthreads();
  for (uint32_t base = 0; base < ns; base += 1024) {
    const uint32_t i = base + tid;
    const bool valid = i < ns;
    const uint32_t s = valid ? S[i] : 2u;
    const bool dig = valid && s <= 1;
    // last non-digit index <= i (block_incl_max pads with 0: scan i + 1, 0 for digits)
    int32_t lnd = (int32_t)block_incl_max(dig ? 0u : i + 1, reinterpret_cast<uint32_t*>(shi)) - 1;
    lnd = max(lnd, carry_lnd);
    const uint32_t k = dig ? (uint32_t)((int32_t)i - lnd - 1) : 0u;
    const uint64_t cntv = valid ? (dig ? ((uint64_t)(s + 1) << min(k, 22u)) : 1ull) : 0ull;
    uint64_t total;
    const uint64_t incl = block_incl_sum(cntv, sh64, &total);
    const uint64_t pos = carry_pos + incl - cntv;
    spos[tid] = (uint32_t)min<uint64_t>(incl - cntv, 0xffffffffull);
    uint8_t byte = 0;
    if (valid) {
      const uint32_t tok = T[i];
      byte = I[(size_t)(i / kMtfChunk) * 256 + tok];
    }
    sbyte[tid] = byte;
    const uint64_t crsp = carry_rsp_sh;
    __syncthreads();
    if (valid) {
      if (dig) {
        const int32_t rs = lnd + 1;  // the run's first digit
        const uint64_t rsp = rs >= (int32_t)base ? carry_pos + spos[rs - (int32_t)base] : crsp;
        if (k >= 1 && pos - rsp > (1ull << 20)) atomicMin(&err_sh, i);
        if (tid == 1023 || i + 1 == ns) carry_rsp_sh = rsp;
      } else if (pos >= nbmax) {
        atomicMin(&err_sh, i);
      }
    }
    // L bytes of this tile: [carry_pos, carry_pos + total) clipped to nbmax
    const uint64_t t0 = carry_pos, t1 = min<uint64_t>(carry_pos + total, nbmax);
    if (t1 > t0) {
      const uint32_t nval = min(ns - base, 1024u);
      for (uint64_t w = (t0 >> 2) + tid; 4 * w < t1; w += 1024) {
        uint32_t word = 0, have = 0;
        // symbol covering byte max(4w, t0): last j with spos[j] <= rel
        const uint64_t a0 = max<uint64_t>(4 * w, t0);
        uint32_t rel = (uint32_t)(a0 - t0);
        uint32_t lo2 = 0, hi2 = nval;  // spos[lo2] <= rel < spos[hi2]
        while (hi2 - lo2 > 1) {
          const uint32_t mid = (lo2 + hi2) >> 1;
          if (spos[mid] <= rel) lo2 = mid; else hi2 = mid;
        }
        for (uint64_t a = a0; a < 4 * w + 4 && a < t1; a++, rel++) {
          while (lo2 + 1 < nval && spos[lo2 + 1] <= rel) lo2++;
          word |= (uint32_t)sbyte[lo2] << (8 * (a & 3));
          have |= 1u << (a & 3);
        }
        if (have == 0xfu) {
          *reinterpret_cast<uint32_t*>(L + 4 * w) = word;
        } else {
          for (uint32_t x = 0; x < 4; x++)
            if ((have >> x) & 1u) L[4 * w + x] = (uint8_t)(word >> (8 * x));
        }
      }
    }
    carry_pos += total;
    __syncthreads();
    if (tid == 1023) shi[0] = lnd;  // the scan's last entry: the tile's last non-digit
    __syncthreads();
    carry_lnd = shi[0];
    __syncthreads();
  }
  if (tid == 0) {
    uint32_t e = err_sh;
    if (eob_reached && carry_pos > nbmax) e = min(e, ns);
    res[c].err2 = e;
    res[c].nblock = (uint32_t)min<uint64_t>(carry_pos, 0xffffffffull);
  }
}

// ---- stage 2: Q[j] = (i << 8) | L[i] for LF(i) = j (the reference's tt, decompress.c:786-791)
__global__ void __launch_bounds__(1024) k_dec_tt(const uint8_t* __restrict__ lbuf, const uint32_t* __restrict__ slot,
                                                 const DecRes* __restrict__ res, uint32_t nbmax,
                                                 uint32_t* __restrict__ qbuf) {
  __shared__ uint32_t hist[16][256];
  __shared__ uint32_t sh[16];
  const uint32_t b = blockIdx.x, c = slot[b];
  const uint32_t n = res[c].nblock;
  const uint8_t* L = lbuf + (size_t)c * nbmax;
  uint32_t* Q = qbuf + (size_t)b * nbmax;
  const uint32_t tid = threadIdx.x, w = tid >> 6, lane = __lane_id();
  for (uint32_t i = tid; i < 16 * 256; i += 1024) (&hist[0][0])[i] = 0;
  __syncthreads();
  const uint32_t seg = ceil_div(ceil_div(n, 16), 64) * 64;
  const uint32_t lo = min(n, w * seg), hi = min(n, lo + seg);
  for (uint32_t i0 = lo; i0 < hi; i0 += 64) {
    const uint32_t i = i0 + lane;
    const bool in = i < hi;
    const uint32_t d = in ? L[i] : 0u;
    const uint64_t m = match_byte(d, __ballot(in));
    if (in && (m & lanemask_lt()) == 0) hist[w][d] += (uint32_t)__popcll(m);
  }
  __syncthreads();
  uint32_t tot = 0;
  if (tid < 256) {
    for (int k = 0; k < 16; k++) {
      const uint32_t x = hist[k][tid];
      hist[k][tid] = tot;
      tot += x;
    }
  }
  const uint32_t incl = block_incl_sum(tot, sh, (uint32_t*)nullptr);
  if (tid < 256) {
    const uint32_t C = incl - tot;
    for (int k = 0; k < 16; k++) hist[k][tid] += C;
  }
  __syncthreads();
  for (uint32_t i0 = lo; i0 < hi; i0 += 64) {
    const uint32_t i = i0 + lane;
    const bool in = i < hi;
    const uint32_t d = in ? L[i] : 0u;
    const uint64_t m = match_byte(d, __ballot(in));
    if (in) {
      const uint32_t pos = hist[w][d] + (uint32_t)__popcll(m & lanemask_lt());
      Q[pos] = (i << 8) | d;
    }
    if (in && (m & lanemask_lt()) == 0) hist[w][d] += (uint32_t)__popcll(m);
  }
}

// Byte writer for a thread-sequential output run: whole aligned words as 4-byte stores, the
// partial words at either end (shared with other threads) as byte stores.
struct ByteSink {
  uint8_t* base;
  uintptr_t lo;  // address of the first byte this sink writes
  uintptr_t a;   // address of the next byte
  uint32_t acc;
  __device__ void init(uint8_t* p) {
    base = p;
    lo = a = reinterpret_cast<uintptr_t>(p);
    acc = 0;
  }
  __device__ __forceinline__ void put(uint32_t b) {
    acc |= b << (8 * (a & 3));
    if ((a & 3) == 3) {
      const uintptr_t w = a - 3;
      if (w >= lo) {
        *reinterpret_cast<uint32_t*>(w) = acc;
      } else {
        for (uintptr_t q = lo; q <= a; q++) *reinterpret_cast<uint8_t*>(q) = (uint8_t)(acc >> (8 * (q & 3)));
      }
      acc = 0;
    }
    a++;
  }
  __device__ void finish() {
    const uintptr_t w = a & ~(uintptr_t)3;
    for (uintptr_t q = max(w, lo); q < a; q++) *reinterpret_cast<uint8_t*>(q) = (uint8_t)(acc >> (8 * (q & 3)));
  }
};

__device__ __forceinline__ uint32_t rand_flip(const uint32_t* __restrict__ rbits, uint32_t period, uint32_t t) {
  const uint32_t k = t % period;
  return (rbits[k >> 5] >> (k & 31)) & 1u;
}

// ---- stage 3: the walk from origPtr (BZ_GET_FAST), split at a ruling set of rows
__global__ void __launch_bounds__(1024) k_dec_walk(const uint32_t* __restrict__ qbuf, const uint32_t* __restrict__ slot,
                                                   const DecRes* __restrict__ res, uint32_t nbmax,
                                                   const uint32_t* __restrict__ rbits, uint32_t rperiod,
                                                   uint8_t* __restrict__ ybuf, uint32_t* __restrict__ cycle_out) {
  __shared__ uint16_t nx[kMaxSplit];
  __shared__ uint32_t ln[kMaxSplit];
  __shared__ uint32_t of[kMaxSplit];
  __shared__ uint32_t cyc_sh;
  const uint32_t b = blockIdx.x, c = slot[b];
  const uint32_t n = res[c].nblock, o = res[c].origptr;
  const bool rnd = res[c].rand != 0;
  const uint32_t* Q = qbuf + (size_t)b * nbmax;
  uint8_t* Y = ybuf + (size_t)c * nbmax;
  const uint32_t ns = ceil_div(n, kSplit) + 1, start = ns - 1;
  auto slot_of = [&](uint32_t s) { return s == start ? o : s * kSplit; };
  auto is_split = [&](uint32_t j) { return j == o || (j % kSplit) == 0; };
  auto id_of = [&](uint32_t j) { return j == o ? start : j / kSplit; };
  for (uint32_t s = threadIdx.x; s < ns; s += blockDim.x) {
    uint32_t j = slot_of(s), len = 0;
    if (s != start && j >= n) {  // past the rows (n a multiple of the spacing): unused
      nx[s] = (uint16_t)start;
      ln[s] = 0;
      of[s] = ~0u;
      continue;
    }
    do {
      j = Q[j] >> 8;
      len++;
    } while (!is_split(j));
    nx[s] = (uint16_t)id_of(j);
    ln[s] = len;
    of[s] = ~0u;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = start, off = 0;
    for (;;) {
      of[s] = off;
      off += ln[s];
      if (off >= n) break;
      s = nx[s];
      if (s == start) break;
    }
    cyc_sh = min(off, n);
  }
  __syncthreads();
  const uint32_t cyc = cyc_sh;
  for (uint32_t s = threadIdx.x; s < ns; s += blockDim.x) {
    const uint32_t t0 = of[s];
    if (t0 == ~0u) continue;
    const uint32_t len = min(ln[s], cyc - t0);
    uint32_t j = slot_of(s), t = t0;
    ByteSink sink;
    sink.init(Y + t0);
    for (uint32_t k = 0; k < len; k++, t++) {
      const uint32_t e = Q[j];
      j = e >> 8;
      uint32_t y = e & 0xffu;
      if (rnd) y ^= rand_flip(rbits, rperiod, t);
      sink.put(y);
    }
    sink.finish();
  }
  if (cyc < n) {  // the walk repeats its cycle (periodic blocks): y[t] = raw[t mod cyc]
    __threadfence_block();
    __syncthreads();
    for (uint32_t t = cyc + threadIdx.x; t < n; t += blockDim.x) {
      const uint32_t s = t % cyc;
      uint32_t y = Y[s];
      if (rnd) y ^= rand_flip(rbits, rperiod, s) ^ rand_flip(rbits, rperiod, t);
      Y[t] = (uint8_t)y;
    }
  }
  if (threadIdx.x == 0) cycle_out[b] = cyc;
}

// ---- stage 3, L2-local form: a block's walk is spread over many workgroups, and the
// workgroups are dealt XCD by XCD in block order (wgmap), so an XCD works on a few blocks at a
// time and their Q arrays (<= 3.6 MB each) stay in its L2 / the MALL instead of every block's
// random 4-byte loads going to HBM.  Splitters every kSplit2 rows; the chain of segments is
// ranked by pointer jumping in LDS (k_dec_walk_rank).
constexpr uint32_t kSplit2 = 64;
constexpr uint32_t kMaxSplit2 = 900000 / kSplit2 + 2;
constexpr uint32_t kWalkT = 256;
constexpr uint16_t kNil = 0xffffu;
// The segment pass also keeps the first kWalkKeep bytes of its segment (the emitted byte of a
// step is in the same Q word as the next row), so the emit pass copies them instead of walking
// the segment's random Q reads a second time; a segment longer than that (a few percent: the
// mean is kSplit2) walks on from the row kept with it.
constexpr uint32_t kWalkKeep = 256;

struct WalkBlock {
  uint32_t n, o, ns, start;
  __device__ WalkBlock(const DecRes& r) : n(r.nblock), o(r.origptr) {
    ns = ceil_div(n, kSplit2) + 1;
    start = ns - 1;
  }
  __device__ uint32_t slot_of(uint32_t s) const { return s == start ? o : s * kSplit2; }
  __device__ bool is_split(uint32_t j) const { return j == o || (j % kSplit2) == 0; }
  __device__ uint32_t id_of(uint32_t j) const { return j == o ? start : j / kSplit2; }
  __device__ bool dead(uint32_t s) const { return s != start && s * kSplit2 == o; }  // start's own row
};

__global__ void __launch_bounds__(kWalkT) k_dec_walk_seg(const uint32_t* __restrict__ qbuf, const uint32_t* __restrict__ slot,
                                                         const DecRes* __restrict__ res, uint32_t nbmax,
                                                         const uint32_t* __restrict__ wgmap, uint32_t* __restrict__ seg_nx,
                                                         uint32_t* __restrict__ seg_len, uint32_t* __restrict__ keep,
                                                         uint32_t* __restrict__ keep_row) {
  const uint32_t m = wgmap[blockIdx.x];
  if (m == ~0u) return;
  const uint32_t b = m >> 8, s = (m & 255u) * kWalkT + threadIdx.x;
  const WalkBlock W(res[slot[b]]);
  if (s >= W.ns) return;
  const uint32_t* Q = qbuf + (size_t)b * nbmax;
  const size_t si = (size_t)b * kMaxSplit2 + s;
  uint32_t* K = keep + si * (kWalkKeep / 4);
  uint32_t j = W.slot_of(s), len = 0, acc = 0;
  do {
    const uint32_t e = Q[j];
    j = e >> 8;
    if (len < kWalkKeep) {
      acc |= (e & 0xffu) << (8 * (len & 3));
      if ((len & 3) == 3) {
        K[len >> 2] = acc;
        acc = 0;
      }
    }
    len++;
    if (len == kWalkKeep) keep_row[si] = j;
  } while (!W.is_split(j));
  if (len < kWalkKeep && (len & 3)) K[len >> 2] = acc;
  seg_nx[si] = W.id_of(j);
  seg_len[si] = len;
}

__global__ void __launch_bounds__(1024) k_dec_walk_rank(const uint32_t* __restrict__ slot, const DecRes* __restrict__ res,
                                                        const uint32_t* __restrict__ seg_nx,
                                                        const uint32_t* __restrict__ seg_len, uint32_t* __restrict__ seg_off,
                                                        uint32_t* __restrict__ cycle_out) {
  __shared__ uint16_t nx[kMaxSplit2];
  __shared__ uint32_t sum[kMaxSplit2];
  constexpr uint32_t kPer = (kMaxSplit2 + 1023) / 1024;
  const uint32_t b = blockIdx.x;
  const WalkBlock W(res[slot[b]]);
  const uint32_t* gn = seg_nx + (size_t)b * kMaxSplit2;
  const uint32_t* gl = seg_len + (size_t)b * kMaxSplit2;
  // the segments of the start's cycle form a list ending at the one that leads back to start
  for (uint32_t s = threadIdx.x; s < W.ns; s += 1024) {
    const uint32_t x = gn[s];
    nx[s] = (x == W.start || W.dead(s)) ? kNil : (uint16_t)x;
    sum[s] = W.dead(s) ? 0u : gl[s];
  }
  __syncthreads();
  // Wyllie list ranking: sum[s] becomes the length from s to the list end; nodes on other
  // cycles never reach the end (their sums are not used)
  for (int round = 0; round < 15; round++) {
    uint32_t ns_[kPer], nn_[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      const uint32_t s = threadIdx.x + 1024 * k;
      ns_[k] = 0;
      nn_[k] = kNil;
      if (s < W.ns) {
        const uint32_t a = nx[s];
        ns_[k] = sum[s];
        if (a != kNil) {
          ns_[k] += sum[a];
          nn_[k] = nx[a];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      const uint32_t s = threadIdx.x + 1024 * k;
      if (s < W.ns) {
        sum[s] = ns_[k];
        nx[s] = (uint16_t)nn_[k];
      }
    }
    __syncthreads();
  }
  const uint32_t total = sum[W.start];  // the start's cycle length (<= n)
  for (uint32_t s = threadIdx.x; s < W.ns; s += 1024)
    seg_off[(size_t)b * kMaxSplit2 + s] = (nx[s] == kNil && !W.dead(s)) ? total - sum[s] : ~0u;
  if (threadIdx.x == 0) cycle_out[b] = min(total, W.n);
}

__global__ void __launch_bounds__(kWalkT) k_dec_walk_emit(const uint32_t* __restrict__ qbuf, const uint32_t* __restrict__ slot,
                                                          const DecRes* __restrict__ res, uint32_t nbmax,
                                                          const uint32_t* __restrict__ wgmap,
                                                          const uint32_t* __restrict__ seg_len,
                                                          const uint32_t* __restrict__ seg_off,
                                                          const uint32_t* __restrict__ cyc_in,
                                                          const uint32_t* __restrict__ rbits, uint32_t rperiod,
                                                          const uint32_t* __restrict__ keep,
                                                          const uint32_t* __restrict__ keep_row,
                                                          uint8_t* __restrict__ ybuf) {
  const uint32_t m = wgmap[blockIdx.x];
  if (m == ~0u) return;
  const uint32_t b = m >> 8, s = (m & 255u) * kWalkT + threadIdx.x;
  const uint32_t c = slot[b];
  const WalkBlock W(res[c]);
  if (s >= W.ns) return;
  const size_t si = (size_t)b * kMaxSplit2 + s;
  const uint32_t t0 = seg_off[si], cyc = cyc_in[b];
  if (t0 >= cyc) return;
  const bool rnd = res[c].rand != 0;
  const uint32_t len = min(seg_len[si], cyc - t0);
  uint8_t* Y = ybuf + (size_t)c * nbmax;
  uint32_t t = t0;
  ByteSink sink;
  sink.init(Y + t0);
  // the bytes the segment pass kept, then (long segments) the walk from the row kept with them
  const uint32_t* K = keep + si * (kWalkKeep / 4);
  const uint32_t nk = min(len, kWalkKeep);
  for (uint32_t k = 0; k < nk; k += 4) {
    const uint32_t w = K[k >> 2];
#pragma unroll
    for (uint32_t x = 0; x < 4; x++) {
      if (k + x >= nk) break;
      uint32_t y = (w >> (8 * x)) & 0xffu;
      if (rnd) y ^= rand_flip(rbits, rperiod, t);
      sink.put(y);
      t++;
    }
  }
  if (len > kWalkKeep) {
    const uint32_t* Q = qbuf + (size_t)b * nbmax;
    uint32_t j = keep_row[si];
    for (uint32_t k = kWalkKeep; k < len; k++, t++) {
      const uint32_t e = Q[j];
      j = e >> 8;
      uint32_t y = e & 0xffu;
      if (rnd) y ^= rand_flip(rbits, rperiod, t);
      sink.put(y);
    }
  }
  sink.finish();
}

// A walk that closed its cycle early repeats it (periodic blocks): y[t] = raw[t mod cyc].
__global__ void __launch_bounds__(256) k_dec_walk_repeat(const uint32_t* __restrict__ slot, const DecRes* __restrict__ res,
                                                         uint32_t nbmax, const uint32_t* __restrict__ cyc_in,
                                                         const uint32_t* __restrict__ rbits, uint32_t rperiod,
                                                         uint8_t* __restrict__ ybuf) {
  const uint32_t b = blockIdx.y, c = slot[b];
  const uint32_t n = res[c].nblock, cyc = cyc_in[b];
  if (cyc >= n || cyc == 0) return;
  const bool rnd = res[c].rand != 0;
  uint8_t* Y = ybuf + (size_t)c * nbmax;
  for (uint32_t t = cyc + blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
    const uint32_t s = t % cyc;
    uint32_t y = Y[s];
    if (rnd) y ^= rand_flip(rbits, rperiod, s) ^ rand_flip(rbits, rperiod, t);
    Y[t] = (uint8_t)y;
  }
}

// ---- stage 4: un-RLE1 (bzlib.c:531-677) as a 5-state machine
// state s: 0 = after a count byte (or at the block start), 1..3 = current run length, 4 = the
// next byte is a count.  A block that ends in state 4 is corrupt (bzlib.c:627-633).
__device__ __forceinline__ void rle_step(uint32_t& s, uint32_t& cnt, uint32_t x, uint32_t prev) {
  if (s == 4) {
    cnt += x;
    s = 0;
  } else {
    cnt += 1;
    s = (s == 0 || x != prev) ? 1u : s + 1;
  }
}

__device__ __forceinline__ void rle_chunk(uint32_t n, uint32_t tid, uint32_t& lo, uint32_t& hi) {
  const uint32_t cs = ceil_div(ceil_div(n, kRleChunks), 16) * 16;
  lo = min(n, tid * cs);
  hi = min(n, lo + cs);
}

__global__ void __launch_bounds__(kRleChunks) k_dec_rle_scan(const uint8_t* __restrict__ ybuf,
                                                              const uint32_t* __restrict__ slot,
                                                              const DecRes* __restrict__ res, uint32_t nbmax,
                                                              uint32_t* __restrict__ info, uint32_t* __restrict__ btot) {
  __shared__ uint32_t fn[kRleChunks][5];  // (count << 3) | end state, per start state
  const uint32_t b = blockIdx.x, c = slot[b];
  const uint32_t n = res[c].nblock;
  const uint8_t* Y = ybuf + (size_t)c * nbmax;
  uint32_t lo, hi;
  rle_chunk(n, threadIdx.x, lo, hi);
  uint32_t st[5] = {0, 1, 2, 3, 4}, ct[5] = {0, 0, 0, 0, 0};
  uint32_t prev = lo ? Y[lo - 1] : 0u;
  uint32_t i = lo;
  for (; i + 16 <= hi; i += 16) {
    const uint4 q = *reinterpret_cast<const uint4*>(Y + i);
    const uint32_t wv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t x = (wv[k >> 2] >> (8 * (k & 3))) & 0xffu;
#pragma unroll
      for (int s = 0; s < 5; s++) rle_step(st[s], ct[s], x, prev);
      prev = x;
    }
  }
  for (; i < hi; i++) {
    const uint32_t x = Y[i];
#pragma unroll
    for (int s = 0; s < 5; s++) rle_step(st[s], ct[s], x, prev);
    prev = x;
  }
#pragma unroll
  for (int s = 0; s < 5; s++) fn[threadIdx.x][s] = (ct[s] << 3) | st[s];
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0, acc = 0;
    for (uint32_t k = 0; k < kRleChunks; k++) {
      info[(size_t)b * kRleChunks + k] = (acc << 3) | s;
      const uint32_t f = fn[k][s];
      acc += f >> 3;
      s = f & 7u;
    }
    btot[2 * b] = acc;
    btot[2 * b + 1] = s;
  }
}

__device__ __forceinline__ uint32_t gf_mul_d(uint32_t a, uint32_t b) {  // a*b mod P (MSB-first CRC-32)
  uint32_t r = 0;
  for (int i = 31; i >= 0; i--) {
    r = (r & 0x80000000u) ? (r << 1) ^ 0x04C11DB7u : (r << 1);
    if ((b >> i) & 1u) r ^= a;
  }
  return r;
}
__device__ __forceinline__ uint32_t shift8(uint32_t a, const uint32_t* __restrict__ xp2, uint64_t len) {
  // a * x^(8 len) mod P; xp2[k] = x^(8 * 2^k)
  for (int k = 0; len; k++, len >>= 1)
    if (len & 1) a = gf_mul_d(a, xp2[k]);
  return a;
}

__global__ void __launch_bounds__(kRleChunks) k_dec_rle_emit(const uint8_t* __restrict__ ybuf,
                                                              const uint32_t* __restrict__ slot,
                                                              const DecRes* __restrict__ res, uint32_t nbmax,
                                                              const uint32_t* __restrict__ info,
                                                              const uint32_t* __restrict__ btot,
                                                              const uint64_t* __restrict__ boff,
                                                              const uint32_t* __restrict__ crc_table,
                                                              const uint32_t* __restrict__ xp2_g, uint8_t* __restrict__ out,
                                                              uint32_t* __restrict__ bcrc) {
  __shared__ uint32_t tab[4][256];  // tab[k][b]: CRC of byte b followed by k zero bytes (slicing by 4)
  __shared__ uint32_t xp2[48];
  __shared__ uint32_t red[kRleChunks / 64];
  const uint32_t b = blockIdx.x, c = slot[b];
  const uint32_t n = res[c].nblock;
  const uint8_t* Y = ybuf + (size_t)c * nbmax;
  {
    uint32_t v = crc_table[threadIdx.x];
    tab[0][threadIdx.x] = v;
    __syncthreads();
#pragma unroll
    for (int k = 1; k < 4; k++) {
      v = (v << 8) ^ tab[0][v >> 24];
      tab[k][threadIdx.x] = v;
    }
  }
  if (threadIdx.x < 48) xp2[threadIdx.x] = xp2_g[threadIdx.x];
  __syncthreads();
  uint32_t lo, hi;
  rle_chunk(n, threadIdx.x, lo, hi);
  const uint32_t inf = info[(size_t)b * kRleChunks + threadIdx.x];
  const uint32_t off = inf >> 3, total = btot[2 * b];
  uint32_t s = inf & 7u;
  uint32_t prev = lo ? Y[lo - 1] : 0u;
  uint32_t crc = 0, emitted = 0, acc = 0, nacc = 0;  // acc: output bytes not yet in the CRC
  ByteSink sink;
  sink.init(out + boff[b] + off);
  auto emit = [&](uint32_t x) {
    acc = (acc << 8) | x;
    if (++nacc == 4) {
      const uint32_t d = crc ^ acc;
      crc = tab[3][d >> 24] ^ tab[2][(d >> 16) & 255u] ^ tab[1][(d >> 8) & 255u] ^ tab[0][d & 255u];
      nacc = 0;
    }
    sink.put(x);
  };
  auto step = [&](uint32_t x) {
    if (s == 4) {
      for (uint32_t k = 0; k < x; k++) emit(prev);
      emitted += x;
      s = 0;
    } else {
      emit(x);
      emitted++;
      s = (s == 0 || x != prev) ? 1u : s + 1;
    }
    prev = x;
  };
  uint32_t i = lo;
  for (; i + 16 <= hi; i += 16) {  // chunks start 16-byte aligned
    const uint4 q = *reinterpret_cast<const uint4*>(Y + i);
    const uint32_t wv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 16; k++) step((wv[k >> 2] >> (8 * (k & 3))) & 0xffu);
  }
  for (; i < hi; i++) step(Y[i]);
  for (uint32_t k = 0; k < nacc; k++) crc = (crc << 8) ^ tab[0][(crc >> 24) ^ ((acc >> (8 * (nacc - 1 - k))) & 255u)];
  sink.finish();
  uint32_t part = emitted ? shift8(crc, xp2, (uint64_t)(total - off - emitted)) : 0u;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) part ^= (uint32_t)__shfl_xor((int)part, o, 64);
  if (__lane_id() == 0) red[threadIdx.x >> 6] = part;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t x = shift8(0xffffffffu, xp2, total);
    for (uint32_t k = 0; k < kRleChunks / 64; k++) x ^= red[k];
    bcrc[b] = ~x;
  }
}

// Positions t (mod the period) whose byte the randomised-block mask flips: t = A_{k+1} - 2 with
// A the running sum of the reference's random-number table (bzlib_private.h:167-179
// BZ_RAND_*, applied to every byte the walk fetches, count bytes included).
const uint16_t kRNums[512] = {
#include "rnums.inc"
};

}  // namespace

struct DecodeWork {
  uint32_t* rbits = nullptr;
  uint32_t rperiod = 0;
};

static void rand_table(Workspace& ws, uint32_t*& bits, uint32_t& period) {
  uint32_t sum = 0;
  for (int k = 0; k < 512; k++) sum += kRNums[k];
  period = sum;
  const uint32_t words = (sum + 31) / 32;
  std::vector<uint32_t> h(words, 0u);
  uint32_t a = 0;
  for (int k = 0; k < 512; k++) {
    a += kRNums[k];
    const uint32_t t = a - 2;
    h[t >> 5] |= 1u << (t & 31);
  }
  bits = ws.u32("dec_rbits", words);
  HIP_OK(hipMemcpy(bits, h.data(), 4 * words, hipMemcpyHostToDevice));
}

// Decodes the .bz2 stream d_in[0, n) into d_out (capacity out_cap).  Returns BZ_OK when the
// stream ends correctly, else the code BZ2_bzBuffToBuffDecompress returns for it.
int decode_stage(Workspace& ws, const uint8_t* d_in, uint64_t n, uint8_t* d_out, uint64_t out_cap,
                 uint64_t* out_len, DecodeStats* stats, hipStream_t st) {
  *out_len = 0;
  uint64_t produced = 0;
  auto eof_code = [&] { return produced == out_cap ? BZ_OUTBUFF_FULL : BZ_UNEXPECTED_EOF; };
  // header "BZh1".."BZh9" (decompress.c:281-292), checked byte by byte as the input arrives
  uint8_t h[16] = {0};
  const uint64_t hn = std::min<uint64_t>(n, 4);
  if (hn) HIP_OK(hipMemcpyAsync(h, d_in, hn, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  const uint8_t want[3] = {'B', 'Z', 'h'};
  for (uint64_t i = 0; i < hn; i++) {
    if (i < 3 && h[i] != want[i]) return BZ_DATA_ERROR_MAGIC;
    if (i == 3 && (h[3] < '1' || h[3] > '9')) return BZ_DATA_ERROR_MAGIC;
  }
  if (n < 4) return eof_code();
  const uint32_t nbmax = 100000u * (uint32_t)(h[3] - '0');
  const uint64_t nbits = 8 * n;

  std::vector<uint64_t> found;
  find_magics_stage(d_in, n, found, st);
  // reads `len` bytes at byte offset `at` (bounded by the stream)
  auto read_bytes = [&](uint64_t at, uint32_t len, uint8_t* dst) {
    std::fill(dst, dst + len, 0);
    if (at < n) {
      HIP_OK(hipMemcpyAsync(dst, d_in + at, std::min<uint64_t>(len, n - at), hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
    }
  };
  auto bits_at = [&](uint64_t bit, uint32_t k) -> uint64_t {  // k <= 48 bits at `bit`
    uint8_t b[8];
    read_bytes(bit >> 3, 8, b);
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | b[i];
    return (v << (bit & 7)) >> (64 - k);
  };
  // no magic where the previous block ended: the reference compares the header bytes one by
  // one (decompress.c:308-322, 650-660), so the outcome is EOF or a data error
  auto bad_header = [&](uint64_t pos) -> int {
    const uint8_t blk[6] = {0x31, 0x41, 0x59, 0x26, 0x53, 0x59}, eos[6] = {0x17, 0x72, 0x45, 0x38, 0x50, 0x90};
    if (pos + 8 > nbits) return eof_code();
    const uint32_t first = (uint32_t)bits_at(pos, 8);
    const uint8_t* m = first == 0x31 ? blk : first == 0x17 ? eos : nullptr;
    if (!m) return BZ_DATA_ERROR;
    for (int k = 1; k < 6; k++) {
      if (pos + 8 * (k + 1) > nbits) return eof_code();
      if ((uint32_t)bits_at(pos + 8 * k, 8) != m[k]) return BZ_DATA_ERROR;
    }
    return BZ_DATA_ERROR;  // not reached: the scan finds every complete magic
  };

  DecodeWork dw;
  rand_table(ws, dw.rbits, dw.rperiod);
  uint32_t combined = 0;
  uint64_t pos = 32;
  DecodeStats ds{};
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  struct EvGuard {
    hipEvent_t a, b;
    ~EvGuard() {
      (void)hipEventDestroy(a);
      (void)hipEventDestroy(b);
    }
  } evg{e0, e1};
  HIP_OK(hipEventRecord(e0, st));
  int rc = BZ_OK;
  for (;;) {
    auto it = std::lower_bound(found.begin(), found.end(), 2 * pos);
    if (it == found.end() || (*it >> 1) != pos) {
      rc = bad_header(pos);
      break;
    }
    if (*it & 1) {  // end of stream: stored combined CRC (decompress.c:662-680)
      if (pos + 48 + 32 > nbits) {
        rc = eof_code();
        break;
      }
      const uint32_t stored = (uint32_t)bits_at(pos + 48, 32);
      rc = stored == combined ? BZ_OK : BZ_DATA_ERROR;
      break;
    }
    // candidates of this pass: block-kind magics from pos on
    std::vector<uint64_t> cand;
    for (auto q = it; q != found.end() && cand.size() < kBatch; ++q)
      if (!(*q & 1)) cand.push_back(*q >> 1);
    const uint32_t nc = (uint32_t)cand.size();
    const uint32_t symstride = nbmax + 128;
    uint64_t* d_cbit = ws.typed<uint64_t>("dec_cbit", nc);
    uint8_t* lbuf = ws.u8("dec_l", (size_t)nc * nbmax + 64);
    uint16_t* symbuf = ws.u16("dec_sym", (size_t)nc * symstride);
    uint8_t* tokbuf = ws.u8("dec_tok", (size_t)nc * symstride);
    uint8_t* seqbuf = ws.u8("dec_seq", (size_t)nc * 256);
    uint8_t* selbuf = ws.u8("dec_sel", (size_t)nc * kSelCap + 64);
    DecRes* d_res = ws.typed<DecRes>("dec_res", nc);
    HIP_OK(hipMemcpyAsync(d_cbit, cand.data(), 8 * nc, hipMemcpyHostToDevice, st));
    static const bool dbg_on = getenv("BZG_DEC_DEBUG") != nullptr;
    uint64_t* d_dbg = dbg_on ? ws.typed<uint64_t>("dec_dbg", 4 * (size_t)nc) : nullptr;
    k_dec_huff<<<nc, 64, 0, st>>>(d_in, n, d_cbit, nc, nbmax, symstride, symbuf, seqbuf, selbuf, d_res, d_dbg);
    HIP_OK(hipGetLastError());
    if (dbg_on) {
      std::vector<uint64_t> h(4 * (size_t)nc);
      HIP_OK(hipMemcpyAsync(h.data(), d_dbg, 8 * h.size(), hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
      double hc = 0, sc = 0, nsy = 0, nbit = 0;
      for (uint32_t k = 0; k < nc; k++) {
        hc += (double)h[4 * k];
        sc += (double)h[4 * k + 1];
        nsy += (double)h[4 * k + 2];
        nbit += (double)h[4 * k + 3];
      }
      fprintf(stderr, "[bzg decode] %u candidates: header %.0f clk, symbols %.0f clk / %.0f sym = %.1f clk/sym, %.0f bits\n",
              nc, hc / nc, sc / nc, nsy / nc, sc / std::max(nsy, 1.0), nbit / nc);
    }
    std::vector<DecRes> hres(nc);
    HIP_OK(hipMemcpyAsync(hres.data(), d_res, sizeof(DecRes) * nc, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    ds.candidates += nc;
    // the chain of blocks through this pass's candidates; a block whose Huffman phase failed
    // ends it (it still goes through phase 2, whose errors may come first)
    std::vector<uint32_t> chain;
    for (;;) {
      auto ci = std::lower_bound(cand.begin(), cand.end(), pos);
      if (ci == cand.end() || *ci != pos) break;
      const uint32_t k = (uint32_t)(ci - cand.begin());
      chain.push_back(k);
      if (hres[k].status != 0) break;
      pos = hres[k].end_bit;
    }
    uint32_t R = (uint32_t)chain.size();
    int stop = BZ_OK;  // a reason to stop inside this pass's blocks
    if (R) {
      uint32_t* d_slot = ws.u32("dec_slot", R);
      HIP_OK(hipMemcpyAsync(d_slot, chain.data(), 4 * R, hipMemcpyHostToDevice, st));
      // ---- phase 2: inverse MTF and runs -> L
      std::vector<uint32_t> cfirst(R + 1, 0), ccand, cj;
      for (uint32_t r = 0; r < R; r++) {
        const uint32_t nch = ceil_div(hres[chain[r]].nsym, kMtfChunk);
        cfirst[r + 1] = cfirst[r] + nch;
        for (uint32_t j = 0; j < nch; j++) {
          ccand.push_back(chain[r]);
          cj.push_back(j);
        }
      }
      const uint32_t Q = cfirst[R];
      uint32_t* d_cfirst = ws.u32("dec_cfirst", R + 1);
      uint32_t* d_ccand = ws.u32("dec_ccand", Q + 1);
      uint32_t* d_cj = ws.u32("dec_cj", Q + 1);
      uint32_t* permbuf = ws.u32("dec_perm", (size_t)Q * 64 + 64);
      uint8_t* initbuf = ws.u8("dec_init", (size_t)Q * 256 + 256);
      HIP_OK(hipMemcpyAsync(d_cfirst, cfirst.data(), 4 * (R + 1), hipMemcpyHostToDevice, st));
      if (Q) {
        HIP_OK(hipMemcpyAsync(d_ccand, ccand.data(), 4 * Q, hipMemcpyHostToDevice, st));
        HIP_OK(hipMemcpyAsync(d_cj, cj.data(), 4 * Q, hipMemcpyHostToDevice, st));
        k_dec_mtf_sym<<<ceil_div(Q, 64), 64, 0, st>>>(symbuf, symstride, d_ccand, d_cj, Q, d_res, tokbuf, permbuf);
        HIP_OK(hipGetLastError());
      }
      k_dec_mtf_chain<<<R, 256, 0, st>>>(d_slot, d_cfirst, d_res, seqbuf, permbuf, initbuf);
      HIP_OK(hipGetLastError());
      k_dec_expand<<<R, 1024, 0, st>>>(d_slot, d_cfirst, nbmax, symstride, symbuf, tokbuf, initbuf, d_res, lbuf);
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(hres.data(), d_res, sizeof(DecRes) * nc, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
      // outcome of each chain block in stream order: a phase-2 rejection at a symbol the
      // Huffman phase decoded comes first; then the Huffman phase's own failure; then origPtr
      int pending = BZ_OK;
      uint32_t ok = 0;
      for (; ok < R; ok++) {
        const DecRes& d = hres[chain[ok]];
        const bool eob = d.status == 0;
        if (d.err2 < d.nsym || (eob && d.err2 == d.nsym)) {
          pending = BZ_DATA_ERROR;
        } else if (!eob) {
          pending = d.status == BZ_UNEXPECTED_EOF ? 1 : BZ_DATA_ERROR;  // 1: EOF marker
        } else if (d.origptr >= d.nblock) {
          pending = BZ_DATA_ERROR;
        }
        if (pending != BZ_OK) break;
      }
      R = ok;
      if (R) {
        uint32_t* qbuf = ws.u32("dec_q", (size_t)R * nbmax + 16);
        uint32_t* cyc = ws.u32("dec_cyc", R);
        uint32_t* info = ws.u32("dec_info", (size_t)R * kRleChunks);
        uint32_t* btot = ws.u32("dec_btot", 2 * R);
        k_dec_tt<<<R, 1024, 0, st>>>(lbuf, d_slot, d_res, nbmax, qbuf);
        HIP_OK(hipGetLastError());
        // Y overwrites L in place: the walk reads only Q
        static const bool walk1 = getenv("BZG_DEC_WALK1") != nullptr;  // one workgroup per block
        if (walk1) {
          k_dec_walk<<<R, 1024, 0, st>>>(qbuf, d_slot, d_res, nbmax, dw.rbits, dw.rperiod, lbuf, cyc);
          HIP_OK(hipGetLastError());
        } else {
          // workgroups of block b go to XCD b % 8, blocks of an XCD in order
          std::vector<std::vector<uint32_t>> per(kNumXcd);
          for (uint32_t r = 0; r < R; r++) {
            const uint32_t nsp = ceil_div(hres[chain[r]].nblock, kSplit2) + 1;
            for (uint32_t w = 0; w < ceil_div(nsp, kWalkT); w++) per[r % kNumXcd].push_back((r << 8) | w);
          }
          size_t G = 0;
          for (auto& v : per) G = std::max(G, v.size());
          std::vector<uint32_t> wgmap(kNumXcd * G, ~0u);
          for (uint32_t x = 0; x < kNumXcd; x++)
            for (size_t j = 0; j < per[x].size(); j++) wgmap[kNumXcd * j + x] = per[x][j];
          uint32_t* d_wgmap = ws.u32("dec_wgmap", wgmap.size());
          uint32_t* seg_nx = ws.u32("dec_segnx", (size_t)R * kMaxSplit2);
          uint32_t* seg_len = ws.u32("dec_seglen", (size_t)R * kMaxSplit2);
          uint32_t* seg_off = ws.u32("dec_segoff", (size_t)R * kMaxSplit2);
          uint32_t* keep = ws.u32("dec_keep", (size_t)R * kMaxSplit2 * (kWalkKeep / 4));
          uint32_t* keep_row = ws.u32("dec_keeprow", (size_t)R * kMaxSplit2);
          HIP_OK(hipMemcpyAsync(d_wgmap, wgmap.data(), 4 * wgmap.size(), hipMemcpyHostToDevice, st));
          const uint32_t nwg = (uint32_t)wgmap.size();
          k_dec_walk_seg<<<nwg, kWalkT, 0, st>>>(qbuf, d_slot, d_res, nbmax, d_wgmap, seg_nx, seg_len, keep, keep_row);
          HIP_OK(hipGetLastError());
          k_dec_walk_rank<<<R, 1024, 0, st>>>(d_slot, d_res, seg_nx, seg_len, seg_off, cyc);
          HIP_OK(hipGetLastError());
          k_dec_walk_emit<<<nwg, kWalkT, 0, st>>>(qbuf, d_slot, d_res, nbmax, d_wgmap, seg_len, seg_off, cyc,
                                                   dw.rbits, dw.rperiod, keep, keep_row, lbuf);
          HIP_OK(hipGetLastError());
          k_dec_walk_repeat<<<dim3(64, R), 256, 0, st>>>(d_slot, d_res, nbmax, cyc, dw.rbits, dw.rperiod, lbuf);
          HIP_OK(hipGetLastError());
        }
        k_dec_rle_scan<<<R, kRleChunks, 0, st>>>(lbuf, d_slot, d_res, nbmax, info, btot);
        HIP_OK(hipGetLastError());
        std::vector<uint32_t> htot(2 * R);
        HIP_OK(hipMemcpyAsync(htot.data(), btot, 8 * R, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        // output order: block r is written only if every earlier block was; a block that ends
        // in a pending count byte is corrupt (data error once its output fits)
        std::vector<uint64_t> hoff(R);
        uint32_t emit = 0;
        uint64_t acc = produced;
        for (uint32_t r = 0; r < R; r++) {
          if (acc + htot[2 * r] > out_cap) {
            stop = BZ_OUTBUFF_FULL;
            break;
          }
          if (htot[2 * r + 1] == 4) {
            stop = BZ_DATA_ERROR;
            break;
          }
          hoff[r] = acc;
          acc += htot[2 * r];
          emit++;
        }
        if (emit) {
          uint64_t* d_boff = ws.typed<uint64_t>("dec_boff", emit);
          uint32_t* d_bcrc = ws.u32("dec_bcrc", emit);
          HIP_OK(hipMemcpyAsync(d_boff, hoff.data(), 8 * emit, hipMemcpyHostToDevice, st));
          k_dec_rle_emit<<<emit, kRleChunks, 0, st>>>(lbuf, d_slot, d_res, nbmax, info, btot, d_boff,
                                                       ws.crc_table(), ws.xpow2_table(), d_out, d_bcrc);
          HIP_OK(hipGetLastError());
          std::vector<uint32_t> hcrc(emit);
          HIP_OK(hipMemcpyAsync(hcrc.data(), d_bcrc, 4 * emit, hipMemcpyDeviceToHost, st));
          HIP_OK(hipStreamSynchronize(st));
          for (uint32_t r = 0; r < emit; r++) {
            produced += htot[2 * r];
            if (hcrc[r] != hres[chain[r]].crc) {  // bzlib.c: block CRC check after its output
              stop = BZ_DATA_ERROR;
              break;
            }
            combined = ((combined << 1) | (combined >> 31)) ^ hcrc[r];
            ds.blocks++;
          }
        }
      }
      if (stop == BZ_OK && pending != BZ_OK) stop = pending == 1 ? eof_code() : BZ_DATA_ERROR;
    }
    if (stop != BZ_OK) {
      rc = stop;
      break;
    }
  }
  HIP_OK(hipEventRecord(e1, st));
  HIP_OK(hipEventSynchronize(e1));
  (void)hipEventElapsedTime(&ds.total_ms, e0, e1);
  ds.out_bytes = produced;
  if (stats) *stats = ds;
  *out_len = produced;
  return rc;
}

}  // namespace bzg
