// mtf.hip -- stage A6: move-to-front + RUNA/RUNB coding (reference compress.c:93-229).
//
// The reference walks each block once, sequentially.  Here every block is cut into chunks of
// kChunk symbols and the list state is composed between chunks:
//   1. sig(c): the distinct symbols of chunk c in order of last occurrence, most recent first
//      (the MTF list after chunk c is sig(c) followed by the untouched rest of the list);
//   2. one wave per block chains list_{c+1} = sig(c) ++ (list_c minus sig(c)) from the
//      initial list (the in-use bytes ascending, compress.c:124-140);
//   3. every chunk re-runs MTF from its own initial list and writes ranks;
//   4. zero runs (which may span chunks) are written as bijective base-2 RUNA/RUNB digits,
//      least significant first (compress.c:154-168); rank j != 0 becomes j+1; EOB =
//      nInUse+1 closes the block (compress.c:225-226).
#include "stages.h"

namespace bzg {

namespace {
constexpr int kT = 256;
constexpr uint32_t kChunk = 1024;

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

__device__ __forceinline__ uint32_t nsym(uint32_t z) { return z ? 31u - (uint32_t)__builtin_clz(z + 1) : 0u; }

// Visits bytes [lo, hi) of p with aligned 16-byte loads (buffers carry >= 16 B of padding),
// forwards or backwards.  f(i, byte).
template <bool kForward, typename F>
__device__ __forceinline__ void for_bytes(const uint8_t* __restrict__ p, uint32_t lo, uint32_t hi, F f) {
  if (lo >= hi) return;
  if (kForward) {
    for (uint32_t a = lo & ~15u; a < hi; a += 16) {
      const uint4 q = *reinterpret_cast<const uint4*>(p + a);
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint32_t i = a + k;
        if (i >= lo && i < hi) f(i, (w[k >> 2] >> (8 * (k & 3))) & 0xffu);
      }
    }
  } else {
    for (uint32_t a = (hi - 1) & ~15u;; a -= 16) {
      const uint4 q = *reinterpret_cast<const uint4*>(p + a);
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 15; k >= 0; k--) {
        const uint32_t i = a + k;
        if (i >= lo && i < hi) f(i, (w[k >> 2] >> (8 * (k & 3))) & 0xffu);
      }
      if (a <= lo) break;
    }
  }
}

// chunk geometry: block b = blockIdx.y, chunk c = blockIdx.x*kT + threadIdx.x
struct ChunkRef {
  bool valid;
  uint32_t b, c, lo, hi, gidx;  // gidx = global chunk id
};
__device__ __forceinline__ ChunkRef chunk_ref(const uint32_t* __restrict__ boff, const uint32_t* __restrict__ cbase) {
  ChunkRef r;
  r.b = blockIdx.y;
  r.c = blockIdx.x * kT + threadIdx.x;
  const uint32_t n = boff[r.b + 1] - boff[r.b];
  r.valid = r.c * kChunk < n;
  r.lo = boff[r.b] + r.c * kChunk;
  r.hi = r.valid ? min(boff[r.b + 1], r.lo + kChunk) : r.lo;
  r.gidx = cbase[r.b] + r.c;
  return r;
}

// 1. signatures.  One lane per chunk walks its chunk backwards in 16-byte words; the words
// of the next kSigAhead steps are in flight while a word is processed (the walk is otherwise
// bound by the latency of one load per 16 symbols).
constexpr uint32_t kSigAhead = 4;
__global__ void __launch_bounds__(kT) k_sig(const uint8_t* __restrict__ L, const uint32_t* __restrict__ boff,
                                            const uint32_t* __restrict__ cbase, uint8_t* __restrict__ sig,
                                            uint32_t* __restrict__ siglen) {
  const ChunkRef r = chunk_ref(boff, cbase);
  if (!r.valid) return;
  // the signature leaves eight bytes per store (a store per new symbol was most of the
  // kernel's time on high-entropy input: ~250 scattered byte stores per chunk; four bytes per
  // store left ~63; sixteen cost text more in selects than they saved: profiles/r05_ab_sig*)
  uint2* out = reinterpret_cast<uint2*>(sig + (size_t)r.gidx * 256);
  uint64_t acc = 0;
  uint32_t cnt = 0;
  uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;  // seen bytes, in registers
  const uint32_t a_lo = r.lo & ~15u;
  uint32_t a = (r.hi - 1) & ~15u;  // word being processed (walking down to a_lo)
  uint4 q[kSigAhead];
#pragma unroll
  for (uint32_t k = 0; k < kSigAhead; k++) {
    const uint32_t ak = a - 16 * k;
    q[k] = (ak >= a_lo && ak <= a) ? *reinterpret_cast<const uint4*>(L + ak) : make_uint4(0, 0, 0, 0);
  }
  for (;;) {
    const uint4 cur = q[0];
#pragma unroll
    for (uint32_t k = 0; k + 1 < kSigAhead; k++) q[k] = q[k + 1];
    {
      const uint32_t an = a - 16 * kSigAhead;  // the word kSigAhead steps down
      q[kSigAhead - 1] = (a >= a_lo + 16 * kSigAhead) ? *reinterpret_cast<const uint4*>(L + an) : make_uint4(0, 0, 0, 0);
    }
    const uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
    for (int k = 15; k >= 0; k--) {
      const uint32_t i = a + k;
      if (i >= r.lo && i < r.hi) {
        const uint32_t c = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
        const uint64_t bit = 1ull << (c & 63);
        const uint32_t qq = c >> 6;
        const uint64_t sw = qq == 0 ? s0 : qq == 1 ? s1 : qq == 2 ? s2 : s3;
        if (!(sw & bit)) {
          s0 |= qq == 0 ? bit : 0ull;
          s1 |= qq == 1 ? bit : 0ull;
          s2 |= qq == 2 ? bit : 0ull;
          s3 |= qq == 3 ? bit : 0ull;
          acc |= (uint64_t)c << (8 * (cnt & 7u));
          if ((++cnt & 7u) == 0) {
            out[(cnt >> 3) - 1] = make_uint2((uint32_t)acc, (uint32_t)(acc >> 32));
            acc = 0;
          }
        }
      }
    }
    if (a <= a_lo) break;
    a -= 16;
  }
  if (cnt & 7u) out[cnt >> 3] = make_uint2((uint32_t)acc, (uint32_t)(acc >> 32));  // (bytes past cnt: unused)
  siglen[r.gidx] = cnt;
}

// 2. list chaining.  list_{c+1} = sig(c) ++ (list_c - sig(c)) is a composition of maps of the
// form F_s(L) = s ++ (L - s), and F_t(F_s(L)) = F_{t ++ (s - t)}(L): the chain is split into
// kCW segments of chunks, one wave each.  Phase 1: every wave chains its segment from the
// empty list (= the segment's combined signature).  Phase 2: wave 0 chains the kCW segment
// signatures from the block's initial list (the in-use bytes ascending, compress.c:124-140),
// giving each segment's first list.  Phase 3: every wave chains its segment again from that
// list and publishes each chunk's initial list.  Critical path: about 2 nch / kCW + kCW steps
// instead of nch.  A lane holds list positions 4l..4l+3.
constexpr uint32_t kCW = 16;

// list <- sig ++ (list - sig) for the list[0, len) of one wave; sw = this lane's 4 signature
// bytes, sl the signature length.  Returns the new length.
__device__ __forceinline__ uint32_t compose_step(uint8_t* list, uint8_t* nlist, uint32_t* mem, uint32_t len,
                                                 uint32_t sl, uint32_t sw, uint32_t lane) {
  if (lane < 8) mem[lane] = 0;
  wave_sync();
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    if (lane * 4 + k < sl) {
      const uint32_t s = (sw >> (8 * k)) & 0xffu;
      atomicOr(&mem[s >> 5], 1u << (s & 31));
      nlist[lane * 4 + k] = (uint8_t)s;
    }
  }
  wave_sync();
  uint32_t keep = 0;
  uint8_t e[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t pos = lane * 4 + k;
    e[k] = list[pos];
    const bool valid = pos < len && !((mem[e[k] >> 5] >> (e[k] & 31)) & 1u);
    keep |= (valid ? 1u : 0u) << k;
  }
  const uint32_t kc = __builtin_popcount(keep);
  const uint32_t incl = wave_incl_sum(kc);
  uint32_t p = sl + incl - kc;
#pragma unroll
  for (int k = 0; k < 4; k++)
    if ((keep >> k) & 1u) nlist[p++] = e[k];
  wave_sync();
  reinterpret_cast<uint32_t*>(list)[lane] = reinterpret_cast<const uint32_t*>(nlist)[lane];
  wave_sync();
  return sl + (uint32_t)__shfl((int)incl, 63, 64);
}

__global__ void __launch_bounds__(64 * kCW) k_compose(const uint32_t* __restrict__ boff, const uint32_t* __restrict__ cbase,
                                                      const uint32_t* __restrict__ inuse, const uint8_t* __restrict__ sig,
                                                      const uint32_t* __restrict__ siglen, uint32_t* __restrict__ init) {
  __shared__ uint8_t list[kCW][256];
  __shared__ uint8_t nlist[kCW][256];
  __shared__ uint32_t mem[kCW][8];
  __shared__ uint8_t segsig[kCW][256];
  __shared__ uint8_t start[kCW][256];
  __shared__ uint32_t seglen[kCW];
  const uint32_t b = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t n = boff[b + 1] - boff[b];
  const uint32_t nch = ceil_div(n, kChunk);
  const uint32_t per = ceil_div(nch, kCW);
  const uint32_t c0 = min(nch, w * per), c1 = min(nch, c0 + per);
  const uint32_t gb = cbase[b];
  auto chain = [&](bool publish, uint32_t len) {
    // the next chunk's signature is loaded one step ahead
    uint32_t sl_n = c0 < c1 ? siglen[gb + c0] : 0u;
    uint32_t sw_n = c0 < c1 ? reinterpret_cast<const uint32_t*>(sig + (size_t)(gb + c0) * 256)[lane] : 0u;
    for (uint32_t c = c0; c < c1; c++) {
      const uint32_t g = gb + c;
      const uint32_t sl = sl_n, sw = sw_n;
      if (c + 1 < c1) {
        sl_n = siglen[g + 1];
        sw_n = reinterpret_cast<const uint32_t*>(sig + (size_t)(g + 1) * 256)[lane];
      }
      if (publish) reinterpret_cast<uint32_t*>(init + (size_t)g * 64)[lane] = reinterpret_cast<const uint32_t*>(list[w])[lane];
      len = compose_step(list[w], nlist[w], mem[w], len, sl, sw, lane);
    }
    return len;
  };
  // phase 1: the segment's signature
  {
    const uint32_t len = chain(false, 0u);
    reinterpret_cast<uint32_t*>(segsig[w])[lane] = reinterpret_cast<const uint32_t*>(list[w])[lane];
    if (lane == 0) seglen[w] = len;
  }
  // the block's initial list: in-use bytes ascending (every wave needs its length)
  uint32_t nu = 0;
  uint32_t wd = inuse[b * 8 + (lane >> 3)];  // lane covers bytes 4l..4l+3
  uint32_t cnt = 0;
  for (int k = 0; k < 4; k++) cnt += (wd >> ((lane * 4 + k) & 31)) & 1u;
  const uint32_t incl = wave_incl_sum(cnt);
  nu = (uint32_t)__shfl((int)incl, 63, 64);
  __syncthreads();
  // phase 2 (wave 0): each segment's first list
  if (w == 0) {
    uint32_t p = incl - cnt;
    for (int k = 0; k < 4; k++) {
      const uint32_t byte = lane * 4 + k;
      if ((wd >> (byte & 31)) & 1u) list[0][p++] = (uint8_t)byte;
    }
    wave_sync();
    uint32_t len = nu;
    for (uint32_t s = 0; s < kCW; s++) {
      reinterpret_cast<uint32_t*>(start[s])[lane] = reinterpret_cast<const uint32_t*>(list[0])[lane];
      wave_sync();
      len = compose_step(list[0], nlist[0], mem[0], len, seglen[s], reinterpret_cast<const uint32_t*>(segsig[s])[lane], lane);
    }
  }
  __syncthreads();
  // phase 3: publish every chunk's initial list
  reinterpret_cast<uint32_t*>(list[w])[lane] = reinterpret_cast<const uint32_t*>(start[w])[lane];
  wave_sync();
  (void)chain(true, nu);
}

// 3. per-chunk MTF from the chunk's initial list, fused with the chunk's zero-run summary.
// List positions 0..31 live in eight registers (byte k of word w = position 4w+k; SWAR
// search and shift, no memory access); positions 32..87 live in LDS as 14 words laid out
// [word][thread]; positions 88..255 stay in the chunk's initial-list words in global memory
// (`init`, updated in place: no other kernel reads a chunk this kernel owns).  Ranks >= 32 are
// rare (< 0.1% on text) and ranks >= 88 rarer still, so the LDS and global parts are touched by
// few steps of a wave, and the small LDS part lets 5 waves share a SIMD instead of 2 (profiles/r05_ab_mtf.txt).
constexpr int kRegW = 8;  // list words (4 positions each) held in registers
constexpr uint32_t kRowMin = 64;  // chunks with more distinct symbols go to k_mtf_q
constexpr int kLdsW = 22;   // list words below this index live in registers or LDS
constexpr int kListW = 64;  // list words a lane holds (registers + LDS + global)

__global__ void __launch_bounds__(kT) k_mtf_run(const uint8_t* __restrict__ L, const uint32_t* __restrict__ boff,
                                                const uint32_t* __restrict__ cbase, const uint32_t* __restrict__ siglen,
                                                uint32_t* __restrict__ init,
                                                uint8_t* __restrict__ ranks, uint32_t* __restrict__ lead,
                                                uint32_t* __restrict__ trail, uint32_t* __restrict__ inner) {
  __shared__ uint32_t lst[kLdsW - kRegW][kT];
  // rank words of the wave's 64 chunks for one 64-symbol window, [chunk][word] (17: no bank
  // conflicts on the per-lane writes); flushed as 16-byte stores, 4 lanes per chunk
  __shared__ uint32_t stg[kT / 64][64 * 17];
  const ChunkRef r = chunk_ref(boff, cbase);
  const uint32_t t = threadIdx.x, lane = __lane_id();
  uint32_t* sw = stg[t >> 6];
  // chunks with many distinct symbols are left to k_mtf_q (their ranks mostly miss the
  // register words)
  const bool mine = r.valid && siglen[r.gidx] <= kRowMin;
  const uint32_t len = mine ? r.hi - r.lo : 0u;
  uint32_t* const src = init + (size_t)(r.valid ? r.gidx : 0u) * 64;
  uint32_t W[kRegW];
#pragma unroll
  for (int w = 0; w < kRegW; w++) W[w] = src[w];
  for (int w = kRegW; w < kLdsW; w++) lst[w - kRegW][t] = src[w];
  // list word w >= kRegW (LDS below kLdsW, else the chunk's own global words)
  auto lget = [&](uint32_t w) -> uint32_t { return w < (uint32_t)kLdsW ? lst[w - kRegW][t] : src[w]; };
  auto lput = [&](uint32_t w, uint32_t v) {
    if (w < (uint32_t)kLdsW) lst[w - kRegW][t] = v;
    else src[w] = v;
  };
  uint32_t racc = 0;  // 4 ranks packed
  uint32_t ld = 0, z = 0, cnt = 0;
  bool seen = false;
  auto step = [&](uint32_t j, uint32_t c) {
    const uint32_t pat = c * 0x01010101u;
    uint32_t fw = kRegW, fz = 0;
#pragma unroll
    for (int w = kRegW - 1; w >= 0; w--) {
      const uint32_t x = W[w] ^ pat;
      const uint32_t zz = (x - 0x01010101u) & ~x & 0x80808080u;
      if (zz) {
        fw = (uint32_t)w;
        fz = zz;
      }
    }
    uint32_t pos;
    if (fw < (uint32_t)kRegW) {
      pos = fw * 4 + ((uint32_t)__builtin_ctz(fz) >> 3);
    } else {  // beyond the register words: LDS words, 4 loads in flight per step (every
              // block byte is in the list)
      const uint32_t wlim = (uint32_t)kListW;
      uint32_t w = kRegW, x = 0;
      for (; w < wlim; w += 4) {
        uint32_t y[4];
#pragma unroll
        for (int k = 0; k < 4; k++) y[k] = lget(w + k) ^ pat;
        uint32_t hit = 4;
#pragma unroll
        for (int k = 3; k >= 0; k--) {
          const uint32_t zz = (y[k] - 0x01010101u) & ~y[k] & 0x80808080u;
          if (zz) {
            hit = (uint32_t)k;
            x = zz;
          }
        }
        if (hit < 4) {
          w += hit;
          break;
        }
      }
      if (w >= 64) {  // only a corrupt input; keeps the loop finite
        w = 63;
        x = 0x80000000u;
      }
      pos = w * 4 + ((uint32_t)__builtin_ctz(x) >> 3);
    }
    const uint32_t rank = pos;
    racc |= rank << (8 * (j & 3));
    if ((j & 3) == 3 || j + 1 == len) {
      sw[lane * 17 + ((j >> 2) & 15)] = racc;
      racc = 0;
    }
    // zero-run summary (RUNA/RUNB symbols of inner runs are counted here)
    if (rank == 0) {
      z++;
      return;
    } else {
      if (!seen) {
        ld = z;
        seen = true;
      } else {
        cnt += nsym(z);
      }
      z = 0;
      cnt++;
    }
    // move c to the front: positions [0, pos) shift up by one byte
    const uint32_t tw = pos >> 2, tb = pos & 3;
    // word w takes its bytes 0..min(pos - 4w, 3) from the list shifted up by one byte
    // (alignbyte of it and the word below), the rest unchanged (bfi with a byte mask)
    uint32_t carry = W[kRegW - 1] >> 24;  // the byte pushed into the LDS part (pos >= 4 kRegW)
    {
      uint32_t prev = c << 24;
      const int nbits = 8 * (int)(pos + 1);
#pragma unroll
      for (int w = 0; w < kRegW; w++) {
        const uint32_t v = W[w];
        const uint32_t shifted = __builtin_amdgcn_alignbyte(v, prev, 3);
        const uint32_t sb = (uint32_t)min(max(nbits - 32 * w, 0), 32);
        const uint32_t mk = (uint32_t)((0xffffffffull << sb) >> 32);
        W[w] = (shifted & mk) | (v & ~mk);
        prev = v;
      }
    }
    if (tw >= (uint32_t)kRegW) {
      uint32_t w = kRegW;
      for (; w + 4 <= tw; w += 4) {  // 4 loads in flight per step
        uint32_t y[4];
#pragma unroll
        for (int k = 0; k < 4; k++) y[k] = lget(w + k);
#pragma unroll
        for (int k = 0; k < 4; k++) {
          lput(w + k, (y[k] << 8) | carry);
          carry = y[k] >> 24;
        }
      }
      for (; w < tw; w++) {
        const uint32_t v = lget(w);
        lput(w, (v << 8) | carry);
        carry = v >> 24;
      }
      const uint32_t v = lget(tw);
      const uint32_t lowmask = (tb == 3) ? 0xffffffffu : ((1u << (8 * (tb + 1))) - 1u);
      lput(tw, (v & ~lowmask) | (((v << 8) | carry) & lowmask));
    }
  };
  // chunk g's ranks go to ranks[g * kChunk, g * kChunk + len): chunk-aligned, so the wave's
  // lanes complete rank words together and every window goes out as full 64-byte segments
  const uint32_t g0 = (uint32_t)__shfl((int)r.gidx, 0, 64);
  // the next window's 64 bytes are loaded while this one is processed (a lane's loads hit a
  // line of its own, so their latency is exposed unless it overlaps the steps)
  uint4 cur[4], nxt[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    cur[k] = make_uint4(0, 0, 0, 0);
    if (16u * k < len) __builtin_memcpy(&cur[k], L + r.lo + 16 * k, 16);  // unaligned; the column is padded
  }
  for (uint32_t w0 = 0; w0 < kChunk; w0 += 64) {
    if (__ballot(len > w0) == 0) break;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      nxt[k] = make_uint4(0, 0, 0, 0);
      if (w0 + 64 + 16u * k < len) __builtin_memcpy(&nxt[k], L + r.lo + w0 + 64 + 16 * k, 16);
    }
    for (uint32_t jj = 0; jj < 64; jj += 16) {
      const uint32_t j0 = w0 + jj;
      const uint4 q = cur[0];
      cur[0] = cur[1];  // register moves: no dynamic indexing of cur
      cur[1] = cur[2];
      cur[2] = cur[3];
      const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int e = 0; e < 16; e++)
        if (j0 + e < len) step(j0 + e, (wd[e >> 2] >> (8 * (e & 3))) & 0xffu);
    }
    wave_sync();
#pragma unroll
    for (uint32_t s4 = 0; s4 < 4; s4++) {
      const uint32_t cc = (lane >> 2) + 16 * s4, qw = (lane & 3) * 4;
      const uint32_t lc = (uint32_t)__shfl((int)len, (int)cc, 64);
      if (lc > w0 + qw * 4) {
        const uint32_t* rw = sw + cc * 17 + qw;
        *reinterpret_cast<uint4*>(ranks + (size_t)(g0 + cc) * kChunk + w0 + qw * 4) = make_uint4(rw[0], rw[1], rw[2], rw[3]);
      }
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < 4; k++) cur[k] = nxt[k];
  }
  if (!mine) return;
  lead[r.gidx] = seen ? ld : 0xffffffffu;  // all-zero chunk marker
  trail[r.gidx] = z;
  inner[r.gidx] = cnt;
}

// Chunks with more than kRowMin distinct symbols (high-entropy blocks: most ranks lie past
// k_mtf_run's register words, where its list search and shift walk LDS word by word), listed
// as (block << 11 | chunk).
__global__ void __launch_bounds__(kT) k_mtf_pick(const uint32_t* __restrict__ boff, const uint32_t* __restrict__ cbase,
                                                 const uint32_t* __restrict__ siglen, uint32_t* __restrict__ hi_list,
                                                 uint32_t* __restrict__ n_hi) {
  const ChunkRef r = chunk_ref(boff, cbase);
  const bool hi = r.valid && siglen[r.gidx] > kRowMin;
  const uint32_t p = wave_append(n_hi, hi);
  if (hi) hi_list[p] = (r.b << 11) | r.c;
}

// 4b. per block (one wave): carried zero runs, chunk output offsets, nMTF.  The zero run
// entering chunk c is a reset-and-add scan over the chunks (a chunk with a nonzero rank
// resets it to its trailing zeros, an all-zero chunk adds its length); a chunk's output is
// nsym(run + its leading zeros) + its inner symbols, and the offsets are their prefix sum.
// 64 chunks per step, carries between steps.
__global__ void __launch_bounds__(64) k_rle2_plan(const uint32_t* __restrict__ boff, const uint32_t* __restrict__ cbase,
                                                  const uint32_t* __restrict__ lead, const uint32_t* __restrict__ trail,
                                                  const uint32_t* __restrict__ inner, uint32_t* __restrict__ zin,
                                                  uint32_t* __restrict__ coff, uint32_t* __restrict__ finalrun,
                                                  uint32_t* __restrict__ nmtf) {
  const uint32_t b = blockIdx.x, lane = __lane_id();
  const uint32_t n = boff[b + 1] - boff[b];
  const uint32_t nch = ceil_div(n, kChunk);
  uint32_t zc = 0, oc = 0;  // carried zero run and output offset
  for (uint32_t c0 = 0; c0 < nch; c0 += 64) {
    const uint32_t c = c0 + lane;
    const bool in = c < nch;
    const uint32_t g = cbase[b] + c;
    const uint32_t ld = in ? lead[g] : 0xffffffffu;
    const bool allz = ld == 0xffffffffu;
    // (reset, value): all-zero chunk adds its length, others reset to their trailing zeros
    uint32_t rs = (in && !allz) ? 1u : 0u;
    uint32_t v = !in ? 0u : allz ? (c + 1 < nch ? kChunk : n - c * kChunk) : trail[g];
    const uint32_t inr = (in && !allz) ? inner[g] : 0u;
    // inclusive scan of the transforms: f2 after f1 = r2 ? (1, v2) : (r1, v1 + v2)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t pr = (uint32_t)__shfl_up((int)rs, o, 64), pv = (uint32_t)__shfl_up((int)v, o, 64);
      if (lane >= (uint32_t)o && !rs) {
        rs = pr;
        v += pv;
      }
    }
    // run after this chunk = rs ? v : zc + v; the run entering it is the previous lane's
    const uint32_t after = rs ? v : zc + v;
    uint32_t before = (uint32_t)__shfl_up((int)after, 1, 64);
    if (lane == 0) before = zc;
    const uint32_t z = before + (allz ? 0u : ld);
    const uint32_t out = (in && !allz) ? nsym(z) + inr : 0u;
    uint32_t incl = out;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = (uint32_t)__shfl_up((int)incl, o, 64);
      if (lane >= (uint32_t)o) incl += x;
    }
    if (in) {
      coff[g] = oc + incl - out;
      zin[g] = allz ? 0u : z;
    }
    zc = (uint32_t)__shfl((int)after, 63, 64);
    oc += (uint32_t)__shfl((int)incl, 63, 64);
  }
  if (lane == 0) {
    finalrun[b] = zc;
    nmtf[b] = oc + nsym(zc) + 1;  // final run + EOB, emitted by the last chunk
  }
}

// 4c. emission + symbol frequencies: one wave per chunk, lane l owns ranks [16l, 16l+16).
// The zero run that ends at a lane's first nonzero rank started in an earlier lane (or chunk:
// zin) -- its length comes from a segmented scan over the lanes.  Each lane writes its
// symbols contiguously at an offset from a wave scan of the per-lane symbol counts.
// MTF of one high-entropy chunk by a quad of lanes (16 chunks per wave), ranks from occurrence
// times (a 16-lane row shifting the list in registers, k_mtf_row, was 1.9x slower: round 4), with the per-chunk state small enough for 64
// chunks per workgroup: lane q keeps the last-occurrence markers of steps 256 q .. 256 q + 255
// (four 64-bit words and their counts) and the used initial-list positions 64 q .. 64 q + 63.
// With m symbols used so far, a symbol last seen at step t has rank m - #{markers <= t}; a
// first occurrence at initial position p has rank m + p - #{used positions < p}.  The symbols
// stream from the BWT column 16 at a time (every lane of the quad loads the same 16 bytes, one
// group ahead); the ranks of 16 steps leave as one 16-byte store; the zero-run summary is kept
// on the way.  Per-chunk LDS: one u16 per byte, its last step or (before its first occurrence)
// 0x8000 | its initial position: 32 KB per workgroup, and at most 128 VGPRs (a few spills per
// 16 steps), so 4 waves share a SIMD instead of 3 (config 5 MTF 63.0 -> 57.6 ms,
// profiles/r05_ab_mtfq_pack.txt).
constexpr uint32_t kQChunks = kT / 4;
__global__ void __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(4))) k_mtf_q(const uint8_t* __restrict__ L, const uint32_t* __restrict__ boff,
                                              const uint32_t* __restrict__ cbase, const uint32_t* __restrict__ init,
                                              const uint32_t* __restrict__ hi_list, const uint32_t* __restrict__ n_hi,
                                              uint8_t* __restrict__ ranks, uint32_t* __restrict__ lead,
                                              uint32_t* __restrict__ trail, uint32_t* __restrict__ inner) {
  // u16 per byte: its last step, or (never seen in the chunk) 0x8000 | its initial position
  __shared__ uint32_t lastw[kQChunks][128];
  const uint32_t nh = *n_hi;
  if (blockIdx.x * kQChunks >= nh) return;
  const uint32_t q = threadIdx.x & 3u, ci = threadIdx.x >> 2;
  const uint32_t i = blockIdx.x * kQChunks + ci;
  const bool valid = i < nh;
  uint32_t len = 0, lo = 0, g = 0;
  if (valid) {
    const uint32_t e = hi_list[i], b = e >> 11, c = e & 2047u;
    lo = boff[b] + c * kChunk;
    len = min(boff[b + 1], lo + kChunk) - lo;
    g = cbase[b] + c;
  }
  uint16_t* last = reinterpret_cast<uint16_t*>(lastw[ci]);
  for (uint32_t k = q; k < 128; k += 4) lastw[ci][k] = 0xffffffffu;
  __builtin_amdgcn_wave_barrier();
  // initial positions, smallest first: lane r writes its 64 positions high to low in round
  // 3 - r, so the lowest lane writes last (past nInUse the list is unspecified)
  {
    uint32_t w[16];
    const uint4* src = reinterpret_cast<const uint4*>(init + (size_t)(valid ? g : 0u) * 64 + 16 * q);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint4 v = src[k];
      w[4 * k] = v.x, w[4 * k + 1] = v.y, w[4 * k + 2] = v.z, w[4 * k + 3] = v.w;
    }
    for (uint32_t r = 0; r < 4; r++) {
      if (q == 3 - r) {
#pragma unroll
        for (int k = 63; k >= 0; k--) last[(w[k >> 2] >> (8 * (k & 3))) & 0xffu] = (uint16_t)(0x8000u | (64 * q + k));
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  __syncthreads();
  uint32_t wl = len;  // the wave runs to its longest chunk
#pragma unroll
  for (int o = 4; o < 64; o <<= 1) wl = max(wl, (uint32_t)__shfl_xor((int)wl, o, 64));
  uint64_t M[4] = {0, 0, 0, 0};   // markers of steps 256 q + 64 w + b
  uint32_t nm[4] = {0, 0, 0, 0};  // their counts per word
  uint64_t S = 0;                 // used initial positions 64 q + b
  uint32_t ns = 0;                // their count
  uint32_t m = 0;                 // symbols used so far
  uint32_t ld = 0, z = 0, cnt = 0;
  bool seen = false;
  auto quad_sum = [](uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    return x;
  };
  const uint8_t* col = L + lo;
  uint4 nxt;
  __builtin_memcpy(&nxt, col, 16);  // (the column is padded)
  uint8_t* rout = ranks + (size_t)(valid ? g : 0u) * kChunk;
  // (steps past wl are inactive like those past len: the 16 steps of a group unroll to
  // straight-line code, all per-lane choices as selects)
  for (uint32_t j16 = 0; j16 < wl; j16 += 16) {
    const uint4 cur = nxt;
    if (j16 + 16 < wl) __builtin_memcpy(&nxt, col + j16 + 16, 16);
    const uint32_t cw[4] = {cur.x, cur.y, cur.z, cur.w};
    uint32_t racc[4] = {0, 0, 0, 0};
    const uint32_t setl = j16 >> 8, setw = (j16 >> 6) & 3u;  // the group's steps share lane and word
#pragma unroll
    for (uint32_t u = 0; u < 16; u++) {
      const uint32_t j = j16 + u;
      const bool act = j < len;
      const uint32_t c = (cw[u >> 2] >> (8 * (u & 3))) & 0xffu;
      const uint32_t t = last[c], p = t & 0xffu;
      const bool first = t >= 0x8000u;
      // this lane's part of #{markers <= t} and of #{used positions < p}
      const uint32_t tl = t >> 8, tw = (t >> 6) & 3u, tb = t & 63u;
      uint64_t mt = M[0];
      mt = tw == 1 ? M[1] : mt;
      mt = tw == 2 ? M[2] : mt;
      mt = tw == 3 ? M[3] : mt;
      const uint32_t below = (tw > 0 ? nm[0] : 0u) + (tw > 1 ? nm[1] : 0u) + (tw > 2 ? nm[2] : 0u);
      const uint32_t xin = below + (uint32_t)__builtin_popcountll(mt & (~0ull >> (63u - tb)));  // bits 0..tb
      const uint32_t nall = nm[0] + nm[1] + nm[2] + nm[3];
      const uint32_t x = q < tl ? nall : (q == tl ? xin : 0u);
      const uint32_t pl = p >> 6, pb = p & 63u;
      const uint32_t yin = (uint32_t)__builtin_popcountll(S & ((1ull << pb) - 1ull));
      const uint32_t y = q < pl ? ns : (q == pl ? yin : 0u);
      const uint32_t tot = quad_sum(first ? y : x);
      const uint32_t rank = first ? m + p - tot : m - tot;
      racc[u >> 2] |= (act ? rank : 0u) << (8 * (u & 3));
      if (act && q == 0) last[c] = (uint16_t)j;
      // the marker moves from step t to step j
      // (the cleared bit is set: an xor; the set word is the group's, a uniform branch)
      const bool clr = act && !first && q == tl;
      const uint64_t bt = clr ? 1ull << tb : 0ull;
#pragma unroll
      for (uint32_t w = 0; w < 4; w++) {
        const bool cw_ = tw == w;
        M[w] ^= cw_ ? bt : 0ull;
        nm[w] -= (cw_ && clr) ? 1u : 0u;
      }
      if (act && q == setl) {
        const uint64_t bj = 1ull << ((j16 & 63u) + u);
        if (setw == 0) {
          M[0] |= bj;
          nm[0]++;
        } else if (setw == 1) {
          M[1] |= bj;
          nm[1]++;
        } else if (setw == 2) {
          M[2] |= bj;
          nm[2]++;
        } else {
          M[3] |= bj;
          nm[3]++;
        }
      }
      const bool fs = act && first && q == pl;
      S = fs ? (S | (1ull << pb)) : S;
      ns += fs ? 1u : 0u;
      m += (act && first) ? 1u : 0u;
      // zero-run summary (the walk of k_mtf_run)
      const bool zr = rank == 0;
      const uint32_t ns_ = seen ? nsym(z) : 0u;
      const uint32_t z2 = zr ? z + 1 : 0u;
      const uint32_t c2 = zr ? cnt : cnt + ns_ + 1u;
      const uint32_t l2 = (!zr && !seen) ? z : ld;
      z = act ? z2 : z;
      cnt = act ? c2 : cnt;
      ld = act ? l2 : ld;
      seen = seen || (act && !zr);
    }
    if (valid && q == 0 && j16 < len) *reinterpret_cast<uint4*>(rout + j16) = make_uint4(racc[0], racc[1], racc[2], racc[3]);
  }
  if (valid && q == 0) {
    lead[g] = seen ? ld : 0xffffffffu;
    trail[g] = z;
    inner[g] = cnt;
  }
}

constexpr int kEW = 16;  // chunks (waves) per workgroup: one frequency flush per 16 chunks
__global__ void __launch_bounds__(64 * kEW) k_rle2_emit(const uint8_t* __restrict__ ranks,
                                                        const uint32_t* __restrict__ boff,
                                                        const uint32_t* __restrict__ cbase,
                                                        const uint32_t* __restrict__ ninuse,
                                                        const uint32_t* __restrict__ zin,
                                                        const uint32_t* __restrict__ coff,
                                                        const uint32_t* __restrict__ finalrun,
                                                        const uint32_t* __restrict__ mtf_off,
                                                        uint16_t* __restrict__ mtfv, uint32_t* __restrict__ freq) {
  // 4 bank-spread copies of every symbol counter (lane & 3 picks one): the ranks are skewed
  // towards 1..3, so one copy made the lanes of a wave queue on a few LDS words
  __shared__ uint32_t hist[kMaxAlpha * 4];
  // the chunk's symbols (<= kChunk ranks + carried-in and final runs + EOB), written out
  // coalesced once the wave has placed them
  __shared__ uint16_t stage[kEW][kChunk + 96];
  for (int i = threadIdx.x; i < kMaxAlpha * 4; i += 64 * kEW) hist[i] = 0;
  __syncthreads();
  const uint32_t b = blockIdx.y, lane = __lane_id();
  uint16_t* st = stage[threadIdx.x >> 6];
  const uint32_t c = blockIdx.x * kEW + (threadIdx.x >> 6);
  const uint32_t n = boff[b + 1] - boff[b];
  if (c * kChunk < n) {
    const uint32_t lo = boff[b] + c * kChunk, hi = min(boff[b + 1], lo + kChunk);
    const uint32_t g = cbase[b] + c;
    const uint32_t base = lo + lane * 16;
    // every load the chunk needs, issued before any is used
    const uint4 q = *reinterpret_cast<const uint4*>(ranks + (size_t)g * kChunk + lane * 16);
    const uint32_t zin_g = zin[g], coff_g = coff[g], fr = finalrun[b], moff_b = mtf_off[b], eob = ninuse[b] + 1;
    uint32_t rk[16];
    uint32_t nzmask = 0;
    {  // chunk-aligned ranks (k_mtf_run): one 16-byte load per lane
      const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 16; k++) rk[k] = base + k < hi ? (wd[k >> 2] >> (8 * (k & 3))) & 0xffu : 0u;
    }
#pragma unroll
    for (int k = 0; k < 16; k++)
      if (base + k < hi && rk[k]) nzmask |= 1u << k;
    const uint32_t cnt = base < hi ? min(16u, hi - base) : 0u;
    const bool has = nzmask != 0;
    const uint32_t lz = has ? (uint32_t)__builtin_ctz(nzmask) : cnt;
    const uint32_t last_nz = has ? 31u - (uint32_t)__builtin_clz(nzmask) : 0u;
    const uint32_t tz = has ? cnt - 1 - last_nz : cnt;
    // zeros carried into each lane: a scan over the lanes that restarts at lanes with a
    // nonzero rank (lane value: has ? trailing zeros : all its zeros)
    uint32_t fl = has ? 1u : 0u, val = has ? tz : cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t pf = (uint32_t)__shfl_up((int)fl, o, 64);
      const uint32_t pv = (uint32_t)__shfl_up((int)val, o, 64);
      if (lane >= (uint32_t)o && !fl) {
        val += pv;
        fl = pf;
      }
    }
    uint32_t cin = (uint32_t)__shfl_up((int)val, 1, 64);
    uint32_t cfl = (uint32_t)__shfl_up((int)fl, 1, 64);
    if (lane == 0) cin = cfl = 0;
    // the run before the chunk's first nonzero rank is zin (it includes the chunk's leading
    // zeros, k_rle2_plan); later runs end inside the chunk
    const uint32_t run0 = cfl ? cin + lz : zin_g;
    uint32_t ecount = 0;
    if (has) {
      ecount += nsym(run0);
      uint32_t zz = 0;
      bool first = true;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        if ((uint32_t)k < cnt) {
          if (rk[k] == 0) {
            zz++;
          } else {
            if (!first) ecount += nsym(zz);
            first = false;
            zz = 0;
            ecount++;
          }
        }
      }
    }
    const bool lastchunk = hi == boff[b + 1];
    const uint32_t tail = (lastchunk && lane == 63) ? nsym(fr) + 1 : 0u;  // final run + EOB
    const uint32_t tot = ecount + tail;
    const uint32_t incl = wave_incl_sum(tot), excl = incl - tot;
    const uint32_t wtot = (uint32_t)__shfl((int)incl, 63, 64);
    uint16_t* out = st + excl;
    uint32_t o = 0, runa = 0, runb = 0;  // RUNA / RUNB counted in registers
    auto put_run = [&](uint32_t zz) {
      while (zz > 0) {
        zz--;
        const uint32_t d = zz & 1u;
        out[o++] = (uint16_t)d;
        runa += d ^ 1u;
        runb += d;
        zz >>= 1;
      }
    };
    if (has) {
      uint32_t zz = 0;
      bool first = true;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        if ((uint32_t)k < cnt) {
          if (rk[k] == 0) {
            zz++;
          } else {
            put_run(first ? run0 : zz);
            first = false;
            zz = 0;
            out[o++] = (uint16_t)(rk[k] + 1);
            atomicAdd(&hist[(rk[k] + 1) * 4 + (lane & 3u)], 1u);
          }
        }
      }
    }
    if (tail) {
      put_run(fr);
      out[o++] = (uint16_t)eob;
      atomicAdd(&hist[eob * 4], 1u);
    }
    if (runa) atomicAdd(&hist[0 * 4 + (lane & 3u)], runa);
    if (runb) atomicAdd(&hist[1 * 4 + (lane & 3u)], runb);
    __builtin_amdgcn_wave_barrier();
    uint16_t* gout = mtfv + moff_b + coff_g;
    for (uint32_t i = lane; i < wtot; i += 64) gout[i] = st[i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kMaxAlpha; i += 64 * kEW) {
    const uint4 c4 = reinterpret_cast<const uint4*>(hist)[i];
    const uint32_t c = c4.x + c4.y + c4.z + c4.w;
    if (c) atomicAdd(&freq[(size_t)b * kMaxAlpha + i], c);
  }
}

}  // namespace

void mtf_stage(Workspace& ws, const Rle1Result& r, const uint8_t* bwt, uint32_t nb, uint32_t total_bytes,
               MtfResult& res, hipStream_t st, const std::vector<uint32_t>* host_boff) {
  (void)total_bytes;
  if (nb == 0) return;
  std::vector<uint32_t> hboff;
  if (host_boff) {
    hboff = *host_boff;
  } else {
    hboff.resize(nb + 1);
    HIP_OK(hipMemcpyAsync(hboff.data(), r.boff, 4 * (nb + 1), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  }
  std::vector<uint32_t> hcb(nb + 1), hmo(nb + 1, 0u);
  uint32_t maxch = 0;
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t nch = ceil_div(hboff[b + 1] - hboff[b], kChunk);
    hcb[b + 1] = hcb[b] + nch;
    maxch = std::max(maxch, nch);
    hmo[b + 1] = (hmo[b] + (hboff[b + 1] - hboff[b]) + 1 + 7) & ~7u;  // nMTF <= n + 1; 16-byte aligned blocks
  }
  const uint32_t nchunks = hcb[nb];
  uint32_t* cbase = ws.u32("mtf_cbase", nb + 1);
  uint32_t* moff = ws.u32("mtf_off", nb + 1);
  HIP_OK(hipMemcpyAsync(cbase, hcb.data(), 4 * (nb + 1), hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync(moff, hmo.data(), 4 * (nb + 1), hipMemcpyHostToDevice, st));
  uint8_t* sig = ws.u8("mtf_sig", (size_t)nchunks * 256);
  uint32_t* siglen = ws.u32("mtf_siglen", nchunks);
  uint32_t* init = ws.u32("mtf_init", (size_t)nchunks * 64);
  uint8_t* ranks = ws.u8("mtf_ranks", (size_t)nchunks * kChunk + 64);  // chunk-aligned
  uint32_t* lead = ws.u32("mtf_lead", nchunks);
  uint32_t* trail = ws.u32("mtf_trail", nchunks);
  uint32_t* inner = ws.u32("mtf_inner", nchunks);
  uint32_t* zin = ws.u32("mtf_zin", nchunks);
  uint32_t* coff = ws.u32("mtf_coff", nchunks);
  uint32_t* finalrun = ws.u32("mtf_final", nb);
  res.nmtf = ws.u32("mtf_n", nb);
  res.freq = ws.u32("mtf_freq", (size_t)nb * kMaxAlpha);
  res.mtfv = ws.u16("mtf_v", hmo[nb] + 16);
  res.mtf_off = moff;
  HIP_OK(hipMemsetAsync(res.freq, 0, (size_t)nb * kMaxAlpha * 4, st));
  const dim3 g2(ceil_div(maxch, kT), nb);
  k_sig<<<g2, kT, 0, st>>>(bwt, r.boff, cbase, sig, siglen);
  HIP_OK(hipGetLastError());
  k_compose<<<nb, 64 * kCW, 0, st>>>(r.boff, cbase, r.inuse, sig, siglen, init);
  HIP_OK(hipGetLastError());
  uint32_t* hi_list = ws.u32("mtf_hilist", nchunks + 16);
  uint32_t* n_hi = ws.u32("mtf_nhi", 16);
  HIP_OK(hipMemsetAsync(n_hi, 0, 4, st));
  k_mtf_pick<<<g2, kT, 0, st>>>(r.boff, cbase, siglen, hi_list, n_hi);
  HIP_OK(hipGetLastError());
  k_mtf_run<<<g2, kT, 0, st>>>(bwt, r.boff, cbase, siglen, init, ranks, lead, trail, inner);
  HIP_OK(hipGetLastError());
  // grid for every chunk; workgroups past the picked count exit at once
  k_mtf_q<<<ceil_div(nchunks, kQChunks), kT, 0, st>>>(bwt, r.boff, cbase, init, hi_list, n_hi, ranks, lead, trail, inner);
  HIP_OK(hipGetLastError());
  k_rle2_plan<<<nb, 64, 0, st>>>(r.boff, cbase, lead, trail, inner, zin, coff, finalrun,
                                                res.nmtf);
  HIP_OK(hipGetLastError());
  k_rle2_emit<<<dim3(ceil_div(maxch, kEW), nb), 64 * kEW, 0, st>>>(ranks, r.boff, cbase, r.ninuse, zin, coff, finalrun,
                                                                   moff, res.mtfv, res.freq);
  HIP_OK(hipGetLastError());
}

}  // namespace bzg
