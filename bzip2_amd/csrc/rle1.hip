// rle1.hip -- stage A1/A2: RLE1, block segmentation, block CRC, in-use maps, period test.
//
// Reference behaviour restated (bzlib.c:211-315 copy_input_until_stop, 361-396
// handle_compress): a run of L equal bytes is cut into chunks of 255 (the last chunk holds
// the remainder); a chunk of 1..3 bytes is copied, a chunk of 4..255 becomes 4 copies plus
// the byte (len-4).  A byte is only consumed while the block holds < nblockMAX bytes, so a
// chunk belongs to the current block iff its first output byte lands before
// blockStart + nblockMAX.  The data-parallel restatement used here:
//   r(i)  = (i - runStart(i)) mod 255          position inside the chunk
//   e(i)  = r<=2 ? 1 : r==3 ? 1+last(i) : last(i)   output bytes produced by input byte i
//   last(i) = chunk ends at i (next byte differs, end of input, or r == 254)
// The output offset of byte i is the exclusive prefix sum of e; a chunk starts at r == 0.
#include "qsa.h"
#include "scan.h"
#include "stages.h"

namespace bzg {

namespace {
constexpr int kT = 256;      // threads
constexpr int kPer = 16;     // bytes per thread
constexpr int kTile = kT * kPer;
static_assert(kT == 256 && kPer == 16, "SWAR fast paths: 4 waves, 4 words per thread");

__device__ __forceinline__ void load16(const uint8_t* __restrict__ x, uint64_t n, uint64_t base,
                                       uint8_t (&v)[kPer]) {
  if (base + kPer <= n && ((base & 15) == 0)) {
    uint4 q = *reinterpret_cast<const uint4*>(x + base);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < kPer; k++) v[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  } else {
#pragma unroll
    for (int k = 0; k < kPer; k++) v[k] = (base + k < n) ? x[base + k] : 0;
  }
}

// Per thread: its run-start bits and whether some byte of it ends a run of 4 (x[i-3..i]
// equal; the 3 bytes before the thread come from one aligned word).  Without such a byte every
// byte of the thread sits at chunk offset r <= 2: it emits itself and starts a chunk iff it
// starts a run, whatever run enters the thread.  On text ~99% of threads are like that.
struct RunBits {
  uint32_t starts;  // bit k: byte base + k starts a run
  uint32_t last1;   // 1 + the thread's last run start (0: none)
  uint32_t nvalid;  // bytes of the thread below n
  bool longrun;
};
__device__ __forceinline__ RunBits run_bits(const uint8_t* __restrict__ x, uint64_t n, uint64_t base,
                                            const uint8_t (&v)[kPer]) {
  uint32_t pw = 0;  // x[base - 4 .. base - 1]; base is a multiple of 16
  if (base >= 4 && base <= n) pw = *reinterpret_cast<const uint32_t*>(x + base - 4);
  uint32_t a3 = (pw >> 8) & 0xffu, a2 = (pw >> 16) & 0xffu, a1 = pw >> 24;  // x[i-3], x[i-2], x[i-1]
  RunBits r{0u, 0u, base < n ? (uint32_t)min<uint64_t>(kPer, n - base) : 0u, false};
  uint32_t lng = 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const uint64_t i = base + k;
    const uint32_t c = v[k];
    const bool ok = i < n;
    if (ok && (i == 0 || c != a1)) {
      r.starts |= 1u << k;
      r.last1 = (uint32_t)i + 1u;
    }
    lng |= (ok && i >= 3 && c == a1 && c == a2 && c == a3) ? 1u : 0u;
    a3 = a2;
    a2 = a1;
    a1 = c;
  }
  r.longrun = lng != 0;
  return r;
}

// The same from the thread's bytes as little-endian words (w: zero past n), pw = the word of
// the 4 bytes before the thread (base >= 4 and base <= n, else unused).
__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[4], int k) { return (w[k >> 2] >> (8 * (k & 3))) & 0xffu; }
__device__ __forceinline__ void load16w(const uint8_t* __restrict__ x, uint64_t n, uint64_t base, uint32_t (&w)[4],
                                        uint32_t& pw) {
  pw = (base >= 4 && base <= n) ? *reinterpret_cast<const uint32_t*>(x + base - 4) : 0u;
  if (base + kPer <= n) {
    const uint4 q = *reinterpret_cast<const uint4*>(x + base);
    w[0] = q.x, w[1] = q.y, w[2] = q.z, w[3] = q.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint32_t a = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) a |= (base + 4 * j + b < n ? (uint32_t)x[base + 4 * j + b] : 0u) << (8 * b);
      w[j] = a;
    }
  }
}
__device__ __forceinline__ RunBits run_bits_words(uint64_t n, uint64_t base, const uint32_t (&w)[4], uint32_t pw) {
  uint32_t a3 = (pw >> 8) & 0xffu, a2 = (pw >> 16) & 0xffu, a1 = pw >> 24;  // x[i-3], x[i-2], x[i-1]
  RunBits r{0u, 0u, base < n ? (uint32_t)min<uint64_t>(kPer, n - base) : 0u, false};
  uint32_t lng = 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const uint64_t i = base + k;
    const uint32_t c = byte_of(w, k);
    const bool ok = i < n;
    if (ok && (i == 0 || c != a1)) {
      r.starts |= 1u << k;
      r.last1 = (uint32_t)i + 1u;
    }
    lng |= (ok && i >= 3 && c == a1 && c == a2 && c == a3) ? 1u : 0u;
    a3 = a2;
    a2 = a1;
    a1 = c;
  }
  r.longrun = lng != 0;
  return r;
}

// SWAR form of run_bits for a thread of a full interior tile (base >= 16, base + 16 < n):
// w = its 16 bytes as little-endian words, pw = the word before them.  Byte k of the thread
// starts a run iff it differs from the byte before; a run of 4 ends at it iff it equals the 3
// bytes before.  Per word: three byte-shifted copies (v_alignbyte), xors, zero-byte masks.
__device__ __forceinline__ uint32_t zero_byte_mask(uint32_t x) {  // 0x80 in every zero byte of x
  return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}
__device__ __forceinline__ uint32_t byte_hi_bits(uint32_t m) {  // bits 7, 15, 23, 31 -> bits 0..3
  return (((m >> 7) * 0x00204081u) >> 21) & 0xfu;
}
struct RunBitsW {
  uint32_t starts;  // bit k: byte k of the thread starts a run
  bool longrun;     // some byte of the thread ends a run of 4
};
__device__ __forceinline__ RunBitsW run_bits_w(const uint32_t (&w)[4], uint32_t pw) {
  uint32_t st = 0, lr = 0, prev = pw;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t p1 = __builtin_amdgcn_alignbyte(w[j], prev, 3);  // bytes i-1
    const uint32_t p2 = __builtin_amdgcn_alignbyte(w[j], prev, 2);  // bytes i-2
    const uint32_t p3 = __builtin_amdgcn_alignbyte(w[j], prev, 1);  // bytes i-3
    const uint32_t d1 = w[j] ^ p1;
    st |= byte_hi_bits(~zero_byte_mask(d1) & 0x80808080u) << (4 * j);
    lr |= zero_byte_mask(d1 | (w[j] ^ p2) | (w[j] ^ p3));
    prev = w[j];
  }
  return RunBitsW{st, lr != 0};
}

// Pass 1: per tile, its last run start (for the carry scan) and its output size up to the
// part that depends on the run entering the tile:  S = output bytes of the bytes from the
// tile's first run start on, h = the bytes before it (they continue the run that starts at the
// carried run start), ends = that run ends at the tile's byte h - 1.  k_rle_fix adds the h
// bytes' output once the carries are known (closed form).  tinfo = S | h << 16 | ends << 31.
// tiles per workgroup of the two RLE1 passes (2 / 4 with all loads in flight: RLE1 +0.36 /
// +0.59 ms per GB, profiles/r05_ab_rle_g.txt)
constexpr uint32_t kRleG = 1;

__device__ __forceinline__ bool rle_interior(uint64_t tile, uint64_t n) {
  return tile > 0 && (tile + 1) * kTile < n;
}

// An interior tile inside one run (config 4): its bytes, the byte before it and the byte
// after it are all equal.  Such a tile starts no run and ends none; every thread must call.
__device__ __forceinline__ bool tile_in_run(const uint8_t* __restrict__ x, uint64_t ts, const uint32_t (&w)[4],
                                            uint32_t pw) {
  const uint32_t c = x[ts], pat = c * 0x01010101u;
  bool ok = w[0] == pat && w[1] == pat && w[2] == pat && w[3] == pat && (pw >> 24) == c;
  if (threadIdx.x == kT - 1) ok = ok && x[ts + kTile] == c;
  return !__syncthreads_or(!ok);
}
// RLE1 output bytes of run offsets [0, x): offsets r mod 255 <= 3 emit the byte, r mod 255 ==
// 254 closes a chunk with its count byte (the closed form of k_rle_fix)
__device__ __forceinline__ uint64_t run_emitted(uint64_t x);

// k_rle_count for one tile that needs the per-byte rules (first, last or run-holding tiles).
// Only threads holding a run of 4 walk their bytes; the others count theirs from the run-start
// bits.  (The bytes are loaded again, as in emit_tile.)
__device__ void rle_count_tile(const uint8_t* __restrict__ x, uint64_t n, uint64_t tile, uint32_t* __restrict__ tmax,
                               uint32_t* __restrict__ tinfo, uint32_t* sh, uint32_t* thr) {
  const uint64_t ts = tile * kTile, base = ts + (uint64_t)threadIdx.x * kPer;
  uint32_t w[4], pw;
  load16w(x, n, base, w, pw);
  const RunBits rb = run_bits_words(n, base, w, pw);
  const uint32_t len = (uint32_t)min<uint64_t>(kTile, n - ts);
  const bool general = __syncthreads_or(rb.longrun);
  const uint32_t incl = block_incl_max(rb.last1, sh);
  if (threadIdx.x == kT - 1) tmax[tile] = incl ? incl - 1u : 0u;
  if (!general) {  // every byte emits itself
    if (threadIdx.x == 0) tinfo[tile] = len;
    return;
  }
  thr[threadIdx.x] = incl;
  __syncthreads();
  uint32_t m1 = threadIdx.x ? thr[threadIdx.x - 1] : 0u;  // 1 + run start of the byte (0: before the tile)
  uint32_t s = 0, h = 0;
  if (!rb.longrun) {
    // bytes before the tile's first run start continue the carried run (h); the rest emit once
    const uint32_t k0 = m1 ? 0u : (rb.starts ? (uint32_t)__builtin_ctz(rb.starts) : (uint32_t)kPer);
    h = min(k0, rb.nvalid);
    s = rb.nvalid - h;
  } else {
    const uint8_t next_after = (base + kPer < n) ? x[base + kPer] : 0;
    uint32_t r = m1 ? ((uint32_t)base - (m1 - 1u)) % 255u : 0u;  // chunk offset carried into byte 0
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint64_t i = base + k;
      if (i >= n) break;
      const uint8_t c = (uint8_t)byte_of(w, k);
      if ((rb.starts >> k) & 1u) {
        m1 = (uint32_t)i + 1u;
        r = 0;
      } else if (k > 0) {
        r = r == 254u ? 0u : r + 1u;
      }
      if (m1 == 0) {
        h++;
      } else {
        const uint8_t nx = (k + 1 < kPer) ? (uint8_t)byte_of(w, k + 1) : next_after;
        const bool last = (i + 1 >= n) || (nx != c) || (r == 254u);
        s += r <= 2u ? 1u : (r == 3u ? 1u + (last ? 1u : 0u) : (last ? 1u : 0u));
      }
    }
  }
  uint32_t tot;
  block_incl_sum(s | (h << 16), sh, &tot);
  if (threadIdx.x == 0) {
    const uint32_t H = tot >> 16;
    const uint32_t ends = (H < len) || (ts + len >= n) || (x[ts + len] != x[ts + len - 1]);
    tinfo[tile] = (tot & 0xffffu) | (H << 16) | (ends << 31);
  }
}

__global__ void __launch_bounds__(kT) BZG_SGPR_LIMIT k_rle_count(const uint8_t* __restrict__ x, uint64_t n, uint64_t tiles,
                                                  uint32_t* __restrict__ tmax, uint32_t* __restrict__ tinfo) {
  __shared__ uint32_t sh[kT / 64];
  __shared__ uint32_t thr[kT];
  const uint64_t t0 = (uint64_t)blockIdx.x * kRleG;
  uint4 q[kRleG];
  uint32_t pw[kRleG];
#pragma unroll
  for (uint32_t g = 0; g < kRleG; g++) {
    const uint64_t base = (t0 + g) * kTile + (uint64_t)threadIdx.x * kPer;
    if (rle_interior(t0 + g, n)) {
      q[g] = *reinterpret_cast<const uint4*>(x + base);
      pw[g] = *reinterpret_cast<const uint32_t*>(x + base - 4);
    }
  }
#pragma unroll
  for (uint32_t g = 0; g < kRleG; g++) {
    const uint64_t tile = t0 + g;
    if (tile >= tiles) break;
    bool done = false;
    if (rle_interior(tile, n)) {  // SWAR run bits first
      const uint32_t w[4] = {q[g].x, q[g].y, q[g].z, q[g].w};
      if (tile_in_run(x, tile * kTile, w, pw[g])) {  // no run start: h = kTile, closed form
        if (threadIdx.x == 0) {
          tmax[tile] = 0;
          tinfo[tile] = (uint32_t)kTile << 16;
        }
        __syncthreads();
        continue;
      }
      const RunBitsW rw = run_bits_w(w, pw[g]);
      if (!__syncthreads_or(rw.longrun)) {  // every byte emits itself: size kTile, last run start
        const uint64_t m = __ballot(rw.starts != 0);
        if (__lane_id() == 0) {
          uint32_t last = 0;
          if (m) {
            const uint32_t l = 63u - (uint32_t)__builtin_clzll(m);
            const uint32_t stl = (uint32_t)__builtin_amdgcn_readlane((int)rw.starts, (int)l);
            last = (uint32_t)(tile * kTile) + (threadIdx.x + l) * kPer + 31u - (uint32_t)__builtin_clz(stl) + 1u;
          }
          sh[threadIdx.x >> 6] = last;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
          const uint32_t a = max(max(sh[0], sh[1]), max(sh[2], sh[3]));
          tmax[tile] = a ? a - 1u : 0u;
          tinfo[tile] = kTile;
        }
        done = true;
      }
    }
    if (!done) rle_count_tile(x, n, tile, tmax, tinfo, sh, thr);
    __syncthreads();  // sh / thr are reused by the next tile
  }
}

// Output bytes of chunk offsets [a, a + h) of one run (r = offset mod 255), the run ending at
// offset a + h - 1 iff `ends`: offsets with r <= 3 emit their byte, r == 254 closes a chunk
// (count byte), and the run's end closes a chunk of 4 or more.
__device__ __forceinline__ uint64_t rle_cnt(uint64_t x, uint32_t lo, uint32_t w) {
  const uint64_t q = x / 255u, r = x % 255u;
  return q * w + (uint64_t)min<uint64_t>(r > lo ? r - lo : 0u, w);
}
__device__ __forceinline__ uint64_t run_emitted(uint64_t x) { return rle_cnt(x, 0, 4) + rle_cnt(x, 254, 1); }

__global__ void k_rle_fix(const uint32_t* __restrict__ carry, const uint32_t* __restrict__ tinfo, uint64_t tiles,
                          uint32_t* __restrict__ tsum) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= tiles) return;
  const uint32_t info = tinfo[t], h = (info >> 16) & 0x1fffu;
  uint64_t e = 0;
  if (h) {
    const uint64_t a = t * kTile - carry[t], b = a + h;
    const uint32_t re = (uint32_t)((b - 1) % 255u);
    e = rle_cnt(b, 0, 4) - rle_cnt(a, 0, 4) + rle_cnt(b, 254, 1) - rle_cnt(a, 254, 1) +
        (((info >> 31) && re >= 3 && re <= 253) ? 1u : 0u);
  }
  tsum[t] = (info & 0xffffu) + (uint32_t)e;
}

struct ByteInfo {
  uint8_t e;  // output bytes
  uint8_t r;  // position inside chunk (0..254)
  bool last;  // chunk ends here
};

// The run start carried into this thread (block max scan over the tile's run starts from the
// tile's carry); every thread of the workgroup must call it.  `thr` needs kT words.
__device__ __forceinline__ uint32_t run_before(uint32_t last_start, uint32_t carry_start, uint32_t* sh,
                                               uint32_t* thr) {
  const uint32_t incl = block_incl_max(last_start, sh);
  thr[threadIdx.x] = incl;
  __syncthreads();
  uint32_t before = carry_start;
  if (threadIdx.x > 0) {
    const uint32_t w = thr[threadIdx.x - 1];
    before = before > w ? before : w;
  }
  __syncthreads();
  return before;
}

// Per-byte info of this thread's 16 bytes given the run start carried into the thread.
__device__ __forceinline__ void byte_info_from(const uint8_t* __restrict__ x, uint64_t n, uint64_t base,
                                               const uint8_t (&v)[kPer], uint32_t before, ByteInfo (&bi)[kPer]) {
  uint8_t prev = (base > 0 && base - 1 < n) ? x[base - 1] : 0;
  uint32_t rs = before;
  const uint8_t next_after = (base + kPer < n) ? x[base + kPer] : 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    uint64_t i = base + k;
    if (i < n && (i == 0 || v[k] != prev)) rs = (uint32_t)i;
    prev = v[k];
    uint32_t r = (uint32_t)(i - rs) % 255u;  // run offsets fit 32 bits (n < 2^32)
    uint8_t nx = (k + 1 < kPer) ? v[k + 1] : next_after;
    bool last = (i + 1 >= n) || (nx != v[k]) || (r == 254);
    uint8_t e = r <= 2 ? 1 : (r == 3 ? (uint8_t)(1 + (last ? 1 : 0)) : (uint8_t)(last ? 1 : 0));
    if (i >= n) e = 0;
    bi[k] = ByteInfo{e, (uint8_t)r, last};
  }
}

// Both of the above (every thread must call it).
__device__ __forceinline__ void byte_info(const uint8_t* __restrict__ x, uint64_t n, uint64_t base,
                                          const uint8_t (&v)[kPer], uint32_t carry_start,
                                          uint32_t* sh, uint32_t* thr, ByteInfo (&bi)[kPer]) {
  uint8_t prev = (base > 0 && base - 1 < n) ? x[base - 1] : 0;
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    uint64_t i = base + k;
    if (i < n && (i == 0 || v[k] != prev)) m = (uint32_t)i;
    prev = v[k];
  }
  byte_info_from(x, n, base, v, run_before(m, carry_start, sh, thr), bi);
}

// Pass 3: write block bytes, chunk-start bitmap and chunk-start -> input position map.
#ifndef BZG_EMIT_WAVES
#define BZG_EMIT_WAVES 0  // 6 or 8: VGPR spills, measured slower (+0.3 / +0.7 ms)
#endif
#ifndef BZG_EMIT_INRUN
#define BZG_EMIT_INRUN 1  // tiles inside one run known from pass 1's tile info: no input read
#endif
#if BZG_EMIT_WAVES > 0
#define BZG_EMIT_BOUNDS __launch_bounds__(kT, BZG_EMIT_WAVES)
#else
#define BZG_EMIT_BOUNDS __launch_bounds__(kT)
#endif
// k_emit for one tile that needs the per-byte rules.  ow / cb: the tile's LDS staging (cb zeroed).
// The thread's 16 bytes are loaded again here (an L2 hit): keeping the words k_emit loaded
// for its fast path alive into this path held the kernel at 86 VGPRs (5 waves per SIMD) against
// 76 (6): RLE1 2.96 -> 2.80 ms per GB (profiles/r05_ab_emit.txt).
__device__ void emit_tile(const uint8_t* __restrict__ x, uint64_t n, uint64_t tile, const uint32_t* __restrict__ carry,
                          const uint32_t* __restrict__ out_base, uint8_t* __restrict__ out,
                          uint32_t* __restrict__ cbits, uint32_t* __restrict__ last_len1, uint32_t* sh, uint32_t* thr,
                          uint32_t* ow, uint32_t* cb) {
  uint8_t* ob = reinterpret_cast<uint8_t*>(ow);
  const uint64_t base = tile * kTile + (uint64_t)threadIdx.x * kPer;
  uint32_t w[4], pw;
  load16w(x, n, base, w, pw);
  const RunBits rb = run_bits_words(n, base, w, pw);
  // per-byte chunk info only for threads holding a run of 4+ (the carry scan only when the
  // tile has one): the others emit their bytes unchanged.  Those threads walk their bytes twice
  // (count, then emit) rather than keeping per-byte info: an array of it held k_emit at 113
  // VGPRs (4 waves per SIMD) for the ~1% of threads that need it.
  uint32_t before = 0;
  if (__syncthreads_or(rb.longrun)) before = run_before(rb.last1 ? rb.last1 - 1u : 0u, carry[tile], sh, thr);
  uint8_t prev0 = 0, next_after = 0;
  uint32_t r0 = 0;
  if (rb.longrun) {
    prev0 = (uint8_t)(pw >> 24);  // (0 at base 0, whose first byte starts a run anyway)
    next_after = (base + kPer < n) ? x[base + kPer] : 0;
    r0 = ((uint32_t)base - before) % 255u;  // chunk offset of the thread's first byte if it continues a run
  }
  // f(k, r, last, e) for the thread's bytes below n: r = chunk offset (0..254), last = the chunk
  // ends here, e = output bytes
  auto walk = [&](auto f) {
    uint8_t prev = prev0;
    uint32_t r = r0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint64_t i = base + k;
      if (i >= n) break;
      const uint8_t c = (uint8_t)byte_of(w, k);
      if (i == 0 || c != prev) r = 0;
      else if (k > 0) r = r == 254u ? 0u : r + 1u;
      prev = c;
      const uint8_t nx = (k + 1 < kPer) ? (uint8_t)byte_of(w, k + 1) : next_after;
      const bool last = (i + 1 >= n) || (nx != c) || (r == 254u);
      const uint32_t e = r <= 2u ? 1u : (r == 3u ? 1u + (last ? 1u : 0u) : (last ? 1u : 0u));
      f(k, i, r, last, e);
    }
  };
  uint32_t s = rb.nvalid;
  if (rb.longrun) {
    s = 0;
    walk([&](int, uint64_t, uint32_t, bool, uint32_t e) { s += e; });
  }
  uint32_t tot;
  uint32_t incl = block_incl_sum(s, sh, &tot);
  const uint32_t t0 = out_base[tile];
  const uint32_t lofs = t0 & 3u;  // LDS byte of output byte p: p - t0 + lofs
  uint32_t pos = t0 + incl - s;
  // chunk-start bits of this thread's outputs span <= 2 words (<= 32 output bytes)
  const uint32_t w0 = pos >> 5;
  uint32_t bits0 = 0, bits1 = 0;
  if (!rb.longrun) {
    const uint32_t sh5 = pos & 31u;
    bits0 = rb.starts << sh5;
    bits1 = sh5 ? rb.starts >> (32u - sh5) : 0u;
    if (base < n && n - base <= kPer) *last_len1 = (rb.starts >> (n - 1 - base)) & 1u;
    if (out != nullptr) {
      const uint32_t lp = pos - t0 + lofs, a = lp & 3u;
      if (rb.nvalid == (uint32_t)kPer && a == 0) {
        uint32_t* o = ow + (lp >> 2);
#pragma unroll
        for (int j = 0; j < 4; j++) o[j] = w[j];
      } else if (rb.nvalid == (uint32_t)kPer) {
        // three whole LDS words in the middle, the bytes of the two edge words (shared with the
        // neighbouring threads) one by one
        uint32_t* o = ow + (lp >> 2);
        for (uint32_t k = 0; k < 4u - a; k++) ob[lp + k] = (uint8_t)byte_of(w, (int)k);
#pragma unroll
        for (int j = 1; j < 4; j++) o[j] = __builtin_amdgcn_alignbyte(w[j], w[j - 1], 4u - a);
        for (uint32_t k = 16u - a; k < 16u; k++) ob[lp + k] = (uint8_t)(w[3] >> (8 * (k & 3u)));
      } else {
#pragma unroll
        for (int k = 0; k < kPer; k++)
          if ((uint32_t)k < rb.nvalid) ob[lp + k] = (uint8_t)byte_of(w, k);
      }
    }
  } else {
    walk([&](int k, uint64_t i, uint32_t r, bool last, uint32_t e) {
      if (i + 1 == n) *last_len1 = (r == 0) ? 1u : 0u;
      if (r == 0) {
        const uint32_t w = pos >> 5;
        if (w == w0) bits0 |= 1u << (pos & 31);
        else bits1 |= 1u << (pos & 31);
      }
      const uint32_t lp = pos - t0 + lofs;
      if (out == nullptr) {  // chunk map only (seg_map_stage): no block bytes
      } else if (r <= 3) {
        ob[lp] = (uint8_t)byte_of(w, k);
        if (r == 3 && last) ob[lp + 1] = 0;
      } else if (last) {
        ob[lp] = (uint8_t)(r - 3);
      }
      pos += e;
    });
  }
  if (bits0) atomicOr(&cb[w0 - (t0 >> 5)], bits0);
  if (bits1) atomicOr(&cb[w0 + 1 - (t0 >> 5)], bits1);
  __syncthreads();
  {  // chunk-start words: the two edge words are shared with the neighbouring tiles
    const uint32_t c0 = t0 >> 5, c1 = tot ? (t0 + tot - 1) >> 5 : c0;
    for (uint32_t q = threadIdx.x; q <= c1 - c0; q += kT) {
      const uint32_t v = cb[q];
      if (q == 0 || q == c1 - c0) {
        if (v) atomicOr(&cbits[c0 + q], v);
      } else {
        cbits[c0 + q] = v;
      }
    }
  }
  if (out == nullptr) return;  // chunk map only (seg_map_stage)
  // output words [t0 / 4, (t0 + tot + 3) / 4): interior ones whole, the two edge words
  // byte by byte (they are shared with the neighbouring tiles)
  const uint32_t nw = (lofs + tot + 3) >> 2;
  uint32_t* outw = reinterpret_cast<uint32_t*>(out) + (t0 >> 2);
  for (uint32_t q = threadIdx.x; q < nw; q += kT) {
    const uint32_t b0 = q * 4, b1 = b0 + 4;
    if (b0 >= lofs && b1 <= lofs + tot) {
      outw[q] = ow[q];
    } else {
      for (uint32_t c = max(b0, lofs); c < min(b1, lofs + tot); c++) out[(t0 & ~3u) + c] = ob[c];
    }
  }
}

// The output of an interior tile inside one run (config 4): the run that started at
// carry[tile] covers the tile, so its output is the run's output from run offset a on: the
// period-5 pattern c c c c 251 (4 bytes and the count byte of each 255-byte chunk), chunk
// starts at pattern phase 0.  The tile's ~80 output bytes are written as whole words (edge
// words, shared with the neighbouring tiles, byte by byte) and its <= 4 chunk-start words
// likewise (edge words with atomicOr).  Words [w_lo, w_hi) of each kind by this thread.
struct RunTile {
  uint32_t c, t0, tot, ph0;
  __device__ uint32_t phase(uint32_t p) const { return (ph0 + (p - t0)) % 5u; }
};
__device__ __forceinline__ RunTile run_tile(const uint8_t* __restrict__ x, uint64_t tile,
                                            const uint32_t* __restrict__ carry, const uint32_t* __restrict__ out_base) {
  const uint64_t a = tile * kTile - carry[tile];
  const uint64_t e0 = run_emitted(a);
  return RunTile{x[tile * kTile], out_base[tile], (uint32_t)(run_emitted(a + kTile) - e0), (uint32_t)(e0 % 5u)};
}
__device__ __forceinline__ void run_tile_word(const RunTile& R, uint8_t* __restrict__ out, uint32_t wi) {
  const uint32_t b0 = wi * 4;
  uint32_t word = 0, inside = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    const uint32_t p = b0 + k;
    if (p >= R.t0 && p < R.t0 + R.tot) {
      word |= (R.phase(p) == 4u ? 251u : R.c) << (8 * k);
      inside++;
    }
  }
  if (inside == 4) {
    reinterpret_cast<uint32_t*>(out)[wi] = word;
  } else {
    for (uint32_t k = 0; k < 4; k++)
      if (b0 + k >= R.t0 && b0 + k < R.t0 + R.tot) out[b0 + k] = (uint8_t)(word >> (8 * k));
  }
}
__device__ __forceinline__ void run_tile_bits(const RunTile& R, uint32_t* __restrict__ cbits, uint32_t cw) {
  const uint32_t c0 = R.t0 >> 5, c1 = (R.t0 + R.tot - 1) >> 5;
  const uint32_t lo = max(cw * 32, R.t0), hi = min(cw * 32 + 32, R.t0 + R.tot);
  uint32_t bits = 0;
  for (uint32_t p = lo; p < hi; p++)
    if (R.phase(p) == 0u) bits |= 1u << (p & 31u);
  if (cw == c0 || cw == c1) {
    if (bits) atomicOr(&cbits[cw], bits);
  } else {
    cbits[cw] = bits;
  }
}
// by the 64 lanes of one wave
__device__ __forceinline__ void emit_run_tile(const uint8_t* __restrict__ x, uint64_t tile,
                                              const uint32_t* __restrict__ carry,
                                              const uint32_t* __restrict__ out_base, uint8_t* __restrict__ out,
                                              uint32_t* __restrict__ cbits, uint32_t lane) {
  const RunTile R = run_tile(x, tile, carry, out_base);
  const uint32_t w0 = R.t0 >> 2, w1 = (R.t0 + R.tot + 3) >> 2;
  if (out != nullptr && lane < w1 - w0) run_tile_word(R, out, w0 + lane);
  const uint32_t c0 = R.t0 >> 5, c1 = (R.t0 + R.tot - 1) >> 5;
  if (lane >= 32 && lane - 32 <= c1 - c0) run_tile_bits(R, cbits, c0 + lane - 32);
}

// Interior tiles inside one run (pass 1's tile info: h = kTile, no run end, S = 0), one thread
// each; k_emit skips them without reading their input.
__global__ void __launch_bounds__(kT) k_emit_runs(const uint8_t* __restrict__ x, uint64_t n, uint64_t tiles,
                                                  const uint32_t* __restrict__ carry,
                                                  const uint32_t* __restrict__ out_base,
                                                  const uint32_t* __restrict__ tinfo, uint8_t* __restrict__ out,
                                                  uint32_t* __restrict__ cbits) {
  const uint64_t tile = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (tile >= tiles || !rle_interior(tile, n) || tinfo[tile] != (uint32_t)kTile << 16) return;
  const RunTile R = run_tile(x, tile, carry, out_base);
  if (out != nullptr)
    for (uint32_t wi = R.t0 >> 2; wi < (R.t0 + R.tot + 3) >> 2; wi++) run_tile_word(R, out, wi);
  for (uint32_t cw = R.t0 >> 5; cw <= (R.t0 + R.tot - 1) >> 5; cw++) run_tile_bits(R, cbits, cw);
}

__global__ void BZG_EMIT_BOUNDS BZG_SGPR_LIMIT k_emit(const uint8_t* __restrict__ x, uint64_t n, uint64_t tiles,
                                             const uint32_t* __restrict__ carry,
                                             const uint32_t* __restrict__ out_base,
                                             uint8_t* __restrict__ out, uint32_t* __restrict__ cbits,
                                             uint32_t* __restrict__ last_len1, const uint32_t* __restrict__ tinfo) {
  __shared__ uint32_t sh[kT / 64];
  __shared__ uint32_t thr[kT];
  // a tile's output (<= 5/4 of its input) staged so that LDS word k is output word
  // (tile start & ~3) / 4 + k; written back with whole-word stores
  __shared__ uint32_t ow[kTile * 5 / 16 + 4];
  __shared__ uint32_t cb[kTile * 5 / 128 + 4];  // chunk-start bits, word k = global word (t0 >> 5) + k
  const uint64_t t0g = (uint64_t)blockIdx.x * kRleG;
  uint4 qs[kRleG];
  uint32_t pws[kRleG], tb[kRleG];
  bool inrun[kRleG];  // pass 1 found the tile inside one run (tinfo: h = kTile, no end, S = 0)
  // the tile's info, output base and input are loaded together (no dependent round trip; an
  // in-run tile's input load is wasted, but such tiles cost nothing else)
#pragma unroll
  for (uint32_t g = 0; g < kRleG; g++) {
    const uint64_t base = (t0g + g) * kTile + (uint64_t)threadIdx.x * kPer;
    const bool interior = rle_interior(t0g + g, n);
    const uint32_t ti = interior ? tinfo[t0g + g] : 0u;
    tb[g] = (t0g + g) < tiles ? out_base[t0g + g] : 0u;
    if (interior) {
      qs[g] = *reinterpret_cast<const uint4*>(x + base);
      pws[g] = *reinterpret_cast<const uint32_t*>(x + base - 4);
    }
    inrun[g] = BZG_EMIT_INRUN && interior && ti == (uint32_t)kTile << 16;
  }
#pragma unroll
  for (uint32_t g = 0; g < kRleG; g++) {
    const uint64_t tile = t0g + g;
    if (tile >= tiles) break;
    if (inrun[g]) continue;  // k_emit_runs (uniform; no LDS touched)
    for (uint32_t i = threadIdx.x; i < kTile * 5 / 128 + 4; i += kT) cb[i] = 0;
    bool done = false;
    if (rle_interior(tile, n)) {  // SWAR run bits first
      const uint4 q = qs[g];
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
      const uint32_t pw = pws[g];
      if (!BZG_EMIT_INRUN && tile_in_run(x, tile * kTile, w, pw)) {
        if (threadIdx.x < 64) emit_run_tile(x, tile, carry, out_base, out, cbits, threadIdx.x);
        __syncthreads();
        continue;
      }
      const RunBitsW rw = run_bits_w(w, pw);
      if (!__syncthreads_or(rw.longrun)) {
        // every byte emits itself and starts a chunk iff it starts a run: the tile's output is
        // its input at t0 = out_base, stored as whole words (the first and last word of the tile
        // are shared with the neighbouring tiles: byte stores)
        const uint32_t t0 = tb[g], lofs = t0 & 3u;
        const uint32_t pos = t0 + threadIdx.x * kPer, sh5 = pos & 31u;
        const uint32_t c0 = t0 >> 5, wi = (pos >> 5) - c0;
        if (rw.starts) {
          atomicOr(&cb[wi], rw.starts << sh5);
          if (sh5 > 16u) atomicOr(&cb[wi + 1], rw.starts >> (32u - sh5));
        }
        uint32_t* outw = reinterpret_cast<uint32_t*>(out) + (pos >> 2);  // word of output byte pos
        if (out != nullptr) {
          if (lofs == 0) {
            *reinterpret_cast<uint4*>(outw) = q;
          } else {
            // output word k of the thread holds the last lofs bytes of input word k - 1 and the
            // first 4 - lofs of word k
            const uint32_t sft = 4u - lofs;
            uint32_t o[5];
            o[0] = __builtin_amdgcn_alignbyte(w[0], pw, sft);
  #pragma unroll
            for (int k = 1; k < 4; k++) o[k] = __builtin_amdgcn_alignbyte(w[k], w[k - 1], sft);
            o[4] = __builtin_amdgcn_alignbyte(0u, w[3], sft);  // the thread's last lofs bytes
            if (threadIdx.x == 0) {
              for (uint32_t c = lofs; c < 4u; c++) out[pos - lofs + c] = (uint8_t)(o[0] >> (8 * c));
            } else {
              outw[0] = o[0];
            }
            outw[1] = o[1];
            outw[2] = o[2];
            outw[3] = o[3];
            if (threadIdx.x == kT - 1)
              for (uint32_t c = 0; c < lofs; c++) out[pos - lofs + 16 + c] = (uint8_t)(o[4] >> (8 * c));
          }
        }
        __syncthreads();
        const uint32_t c1 = (t0 + kTile - 1) >> 5;
        for (uint32_t k = threadIdx.x; k <= c1 - c0; k += kT) {
          const uint32_t b = cb[k];
          if (k == 0 || k == c1 - c0) {
            if (b) atomicOr(&cbits[c0 + k], b);
          } else {
            cbits[c0 + k] = b;
          }
        }
        done = true;
      }
    }
    if (!done) emit_tile(x, n, tile, carry, out_base, out, cbits, last_len1, sh, thr, ow, cb);
    __syncthreads();  // the LDS staging is reused by the next tile
  }
}

// Input offset of the chunk whose first output byte is p (p a chunk start), by re-deriving
// the byte info of the one RLE tile that produced p.  One workgroup per queried boundary.
__global__ void __launch_bounds__(kT) BZG_SGPR_LIMIT k_chunk_inpos(const uint8_t* __restrict__ x, uint64_t n,
                                                    const uint32_t* __restrict__ carry,
                                                    const uint32_t* __restrict__ out_base, uint32_t ntiles,
                                                    const uint32_t* __restrict__ qpos, uint32_t nq,
                                                    uint32_t* __restrict__ inpos) {
  __shared__ uint32_t sh[kT / 64];
  __shared__ uint32_t thr[kT];
  const uint32_t q = blockIdx.x;
  if (q >= nq) return;
  const uint32_t p = qpos[q];
  // tile whose output range contains p: largest t with out_base[t] <= p
  uint32_t lo = 0, hi = ntiles;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (out_base[mid] <= p) lo = mid;
    else hi = mid;
  }
  const uint64_t base = (uint64_t)lo * kTile + (uint64_t)threadIdx.x * kPer;
  uint8_t v[kPer];
  load16(x, n, base, v);
  ByteInfo bi[kPer];
  byte_info(x, n, base, v, carry[lo], sh, thr, bi);
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) s += bi[k].e;
  uint32_t incl = block_incl_sum(s, sh, (uint32_t*)nullptr);
  uint32_t pos = out_base[lo] + incl - s;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    if (base + k >= n) break;
    if (pos == p && bi[k].r == 0) inpos[q] = (uint32_t)(base + k);
    pos += bi[k].e;
  }
}

// Block-cut walk (one wave), for a batch (fill 0) and for one region of a sharded stream
// (SURVEY.md 8e).  The region starts
// at a chunk start of the stream with `fill_in` RLE1 bytes (< nblock_max) already in the open
// block, so the first cut is the first chunk start at output position >= nblock_max - fill_in;
// after that, a cut is the first chunk start >= the previous cut + nblock_max (file header);
// with final_region, the last chunk never starts a block when it is 1 byte (FINISH).  qpos gets the cut positions followed by the region's last
// chunk start; res = {ncuts, last chunk start, open-block fill at that chunk start}.
// A chunk is at most 5 RLE1 bytes, so the cut after s lies in [s + M, s + M + 4] (M =
// nblock_max) and the (j+1)-th cut after s in [s + (j+1) M, s + (j+1) M + 4 j + 4].  Each round,
// lane j loads the <= 10 bitmap words of that window for step j into LDS (all loads in flight
// at once).  The 64 steps are then resolved optimistically: every remaining step is assumed to
// cut exactly M after the previous cut (true whenever a chunk starts there, as on text); a
// ballot finds the first step where that fails, the steps before it are written in parallel,
// and that one step is resolved from its window.
constexpr int kWalkWords = 10;
__global__ void __launch_bounds__(64) k_segment_fill(const uint32_t* __restrict__ cbits,
                                                     const uint32_t* __restrict__ m_ptr, uint32_t nblock_max,
                                                     uint32_t fill_in, int final_region,
                                                     const uint32_t* __restrict__ last_len1_ptr,
                                                     uint32_t* __restrict__ qpos, uint32_t* __restrict__ res,
                                                     uint32_t max_cuts) {
  __shared__ uint32_t win[64][kWalkWords];
  const uint32_t lane = threadIdx.x;
  const uint32_t m = *m_ptr;
  if (m == 0) {
    if (lane == 0) {
      res[0] = res[1] = 0;
      res[2] = fill_in;
      qpos[0] = 0;
    }
    return;
  }
  const uint32_t wend = (m + 31) >> 5;
  const int64_t M = (int64_t)nblock_max;
  uint32_t last_start = 0;  // every lane computes it (uniform)
  {
    uint32_t w = (m - 1) >> 5;
    for (;;) {
      uint32_t bits = cbits[w] & (w == ((m - 1) >> 5) ? (0xffffffffu >> (31 - ((m - 1) & 31))) : ~0u);
      if (bits) { last_start = (w << 5) + 31 - (uint32_t)__builtin_clz(bits); break; }
      if (w == 0) break;
      --w;
    }
  }
  const bool tail_rule = final_region && *last_len1_ptr;
  int64_t s = -(int64_t)fill_in;  // output position of the open block's start (uniform)
  uint32_t b = 0;                 // cuts so far (uniform)
  int done = 0;                   // 1: walk ended, 2: more than max_cuts
  while (!done) {
    {
      const int64_t lo = s + (int64_t)(lane + 1) * M;
      const int64_t w0 = lo < 0 ? 0 : (lo >> 5);
#pragma unroll
      for (int k = 0; k < kWalkWords; k++) {
        const int64_t w = w0 + k;
        win[lane][k] = (w < (int64_t)wend) ? cbits[w] : 0u;
      }
    }
    __syncthreads();
    int64_t cur = s;
    uint32_t j = 0;
    while (j < 64 && !done) {
      bool ok = false;
      int64_t tl = 0;
      if (lane >= j) {
        tl = cur + (int64_t)(lane - j + 1) * M;
        if (tl >= 0 && tl < (int64_t)m && !(tail_rule && tl == (int64_t)last_start) && b + (lane - j) < max_cuts) {
          const int64_t lo = s + (int64_t)(lane + 1) * M;
          const int64_t k = (tl >> 5) - (lo < 0 ? 0 : (lo >> 5));
          ok = k >= 0 && k < kWalkWords && ((win[lane][k] >> (tl & 31)) & 1u);
        }
      }
      const uint64_t bad = __ballot(!ok) & (~0ull << j);
      const uint32_t f = bad ? (uint32_t)__builtin_ctzll(bad) : 64u;
      if (ok && lane < f) qpos[b + (lane - j)] = (uint32_t)tl;
      if (f > j) {
        cur += (int64_t)(f - j) * M;
        b += f - j;
        j = f;
      }
      if (f < 64) {  // step f from its window
        const int64_t lo = s + (int64_t)(f + 1) * M;
        const int64_t w0 = lo < 0 ? 0 : (lo >> 5);
        const int64_t t = cur + M;
        uint32_t p = m;
        if (t <= 0) {
          p = 0;
        } else if (t < (int64_t)m) {
          const int64_t tw = t >> 5;
          for (int64_t w = tw; w < w0 + kWalkWords && w < (int64_t)wend; w++) {
            uint32_t bits = win[f][w - w0];
            if (w == tw) bits &= ~0u << (t & 31);
            if (bits) {
              p = (uint32_t)((w << 5) + __builtin_ctz(bits));
              break;
            }
          }
          if (p > m) p = m;
        }
        if (p < m && tail_rule && p == last_start) p = m;
        if (p >= m) {
          done = 1;
        } else if (b >= max_cuts) {  // cannot happen with the host's sizing; keeps the walk finite
          done = 2;
        } else {
          if (lane == 0) qpos[b] = p;
          b++;
          cur = p;
          j = f + 1;
        }
      }
    }
    __syncthreads();  // the next round overwrites win
    s = cur;
  }
  if (lane == 0) {
    if (done == 2) {
      res[0] = 0xffffffffu;
    } else {
      qpos[b] = last_start;
      res[0] = b;
      res[1] = last_start;
      res[2] = (uint32_t)((int64_t)last_start - s);
    }
  }
}

// Block offsets from k_segment_fill's cuts (written at boff + 1): boff[0] = 0; a final batch
// closes its last block at m, a non-final one leaves the block after the last cut open (it
// restarts the next batch from its input start).
__global__ void k_set_word(uint32_t* __restrict__ p, uint32_t v) {
  if (threadIdx.x == 0) p[0] = v;
}

__global__ void k_segment_finish(const uint32_t* __restrict__ m_ptr, const uint32_t* __restrict__ res,
                                 int final_batch, uint32_t* __restrict__ boff, uint32_t* __restrict__ nblocks) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint32_t m = *m_ptr, ncut = res[0];
  boff[0] = 0;
  if (ncut == 0xffffffffu) {
    *nblocks = 0xffffffffu;
  } else if (m == 0) {
    *nblocks = 0;
  } else if (final_batch) {
    boff[ncut + 1] = m;
    *nblocks = ncut + 1;
  } else {
    *nblocks = ncut;
  }
}

// CRC helpers: MSB-first polynomial 0x04C11DB7.
__device__ __forceinline__ uint32_t gf_mul(uint32_t a, uint32_t b) {  // a*b mod P
  uint32_t r = 0;
  for (int i = 31; i >= 0; i--) {
    r = (r & 0x80000000u) ? (r << 1) ^ 0x04C11DB7u : (r << 1);
    if ((b >> i) & 1u) r ^= a;
  }
  return r;
}
// x^(8*len) mod P via the table of x^(2^k) mod P for k = 3 .. 3+40
__device__ __forceinline__ uint32_t xpow8(const uint32_t* __restrict__ xp2, uint64_t len) {
  uint32_t r = 1u;  // x^0 (bit k of a CRC register is the coefficient of x^k)
  int k = 0;
  while (len) {
    if (len & 1) r = gf_mul(r, xp2[k]);
    len >>= 1;
    ++k;
  }
  return r;
}

// Block CRC over input [binst[b], binst[b+1]).  The CRC without init / final xor is linear:
// crc(A || B) = crc(A) * x^(8|B|) + crc(B) over GF(2).  `split` workgroups per block take
// equal sub-ranges (8 for ordinary blocks; up to kCrcSplitMax for blocks of long runs, whose
// input spans up to 46 MB); in a sub-range, round r gives thread t the 16 bytes at 4096 r + 16 t
// (coalesced loads), whose CRC (slicing by 16, LDS tables) is folded into the thread's
// accumulator as acc = acc * x^(8*4096) + crc(piece) (the multiplication by a constant is a
// linear map: 4 LDS table lookups).  The accumulators are then shifted to their end
// positions and xor-ed; k_crc_combine folds the sub-ranges and the init/final xor.
constexpr uint32_t kCrcSplit = 8;       // sub-ranges per block, at least
constexpr uint32_t kCrcSplitMax = 256;  // and at most (>= 512 KB each in between)
constexpr uint32_t kCrcRound = kT * 16;

__device__ __forceinline__ uint32_t crc_pow_mul(uint32_t a, const uint32_t* __restrict__ xp2, uint64_t len) {
  return len ? gf_mul(a, xpow8(xp2, len)) : a;
}

__global__ void __launch_bounds__(kT) k_block_crc(const uint8_t* __restrict__ x, const uint32_t* __restrict__ binst,
                                                  const uint32_t* __restrict__ crc_table_g,
                                                  const uint32_t* __restrict__ xp2_g, uint32_t split,
                                                  uint32_t* __restrict__ part, const uint32_t* __restrict__ tinfo,
                                                  uint64_t n) {
  __shared__ uint32_t tab[16][256];  // tab[k][b] = crc of byte b followed by k zero bytes
  __shared__ uint32_t mul[4][256];   // byte k of a (from the top) times x^(8*4096)
  __shared__ uint32_t xp2[48];
  __shared__ uint32_t red[kT / 64];
  const uint32_t b = blockIdx.y, w = blockIdx.x;
  if (threadIdx.x < 48) xp2[threadIdx.x] = xp2_g[threadIdx.x];
  {
    uint32_t v = crc_table_g[threadIdx.x];
    tab[0][threadIdx.x] = v;
    __syncthreads();
#pragma unroll
    for (int k = 1; k < 16; k++) {
      v = (v << 8) ^ tab[0][v >> 24];
      tab[k][threadIdx.x] = v;
    }
  }
  __syncthreads();
  {
    const uint32_t xr = xpow8(xp2, kCrcRound);
#pragma unroll
    for (int k = 0; k < 4; k++) mul[k][threadIdx.x] = gf_mul(threadIdx.x << (8 * (3 - k)), xr);
  }
  const uint32_t lo = binst[b], hi = binst[b + 1];
  const uint32_t per = ceil_div(hi - lo, split);
  const uint32_t s0 = min(hi, lo + w * per), s1 = min(hi, s0 + per);
  const uint32_t len = s1 - s0, R = len / kCrcRound, T = len - R * kCrcRound;
  __syncthreads();
  auto crc16q = [&](const uint4 q) {
    const uint32_t a = bswap32(q.x), d1 = bswap32(q.y), d2 = bswap32(q.z), d3 = bswap32(q.w);
    return tab[15][a >> 24] ^ tab[14][(a >> 16) & 255u] ^ tab[13][(a >> 8) & 255u] ^ tab[12][a & 255u] ^
           tab[11][d1 >> 24] ^ tab[10][(d1 >> 16) & 255u] ^ tab[9][(d1 >> 8) & 255u] ^ tab[8][d1 & 255u] ^
           tab[7][d2 >> 24] ^ tab[6][(d2 >> 16) & 255u] ^ tab[5][(d2 >> 8) & 255u] ^ tab[4][d2 & 255u] ^
           tab[3][d3 >> 24] ^ tab[2][(d3 >> 16) & 255u] ^ tab[1][(d3 >> 8) & 255u] ^ tab[0][d3 & 255u];
  };
  auto crc16 = [&](const uint8_t* p) {
    uint4 q;
    __builtin_memcpy(&q, p, 16);
    return crc16q(q);
  };
  auto fold = [&](uint32_t acc, uint32_t c) {
    return mul[0][acc >> 24] ^ mul[1][(acc >> 16) & 255u] ^ mul[2][(acc >> 8) & 255u] ^ mul[3][acc & 255u] ^ c;
  };
  uint32_t acc = 0;
  const uint8_t* px = x + s0 + 16 * threadIdx.x;
  uint32_t r = 0;
  // a sub-range inside one run (its tiles all inside one run by pass 1's tile info, config 4):
  // every round's piece is 16 copies of the run's byte, so the rounds fold without loads
  bool in_run = len > 0;
  for (uint32_t t = s0 / kTile + threadIdx.x; in_run && t <= (s1 - 1) / kTile; t += kT)
    in_run = rle_interior(t, n) && tinfo[t] == (uint32_t)kTile << 16;
  if (!__syncthreads_or(!in_run) && R) {
    const uint32_t pat = x[s0] * 0x01010101u;
    const uint32_t v = crc16q(make_uint4(pat, pat, pat, pat));
    for (; r < R; r++) acc = fold(acc, v);
  }
  // 4 rounds' loads in flight before their folds
  for (; r + 4 <= R; r += 4) {
    uint4 q[4];
#pragma unroll
    for (int k = 0; k < 4; k++) __builtin_memcpy(&q[k], px + (size_t)(r + k) * kCrcRound, 16);
#pragma unroll
    for (int k = 0; k < 4; k++) acc = fold(acc, crc16q(q[k]));
  }
  for (; r < R; r++) acc = fold(acc, crc16(px + (size_t)r * kCrcRound));
  uint32_t res = R ? crc_pow_mul(acc, xp2, kCrcRound - 16 * (threadIdx.x + 1) + T) : 0u;
  // the tail: thread t takes bytes [16 t, 16 t + 16) of it
  const uint32_t tb = 16 * threadIdx.x;
  if (tb < T) {
    const uint32_t m = min(16u, T - tb);
    const uint8_t* pt = x + s0 + R * kCrcRound + tb;
    uint32_t c = 0;
    if (m == 16) {
      c = crc16(pt);
    } else {
      for (uint32_t i = 0; i < m; i++) c = (c << 8) ^ tab[0][(c >> 24) ^ pt[i]];
    }
    res ^= crc_pow_mul(c, xp2, T - tb - m);
  }
  // xor over the workgroup
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) res ^= (uint32_t)__shfl_xor((int)res, o, 64);
  if (__lane_id() == 0) red[threadIdx.x >> 6] = res;
  __syncthreads();
  if (threadIdx.x == 0) part[b * split + w] = red[0] ^ red[1] ^ red[2] ^ red[3];
}

// One wave per block: lane l shifts the CRCs of sub-ranges l, l + 64, ... to the block end,
// lane 63 also the initial register through the whole block; the lanes' terms are xor-ed.
__global__ void __launch_bounds__(64) k_crc_combine(const uint32_t* __restrict__ binst, const uint32_t* __restrict__ part,
                                                    const uint32_t* __restrict__ xp2, uint32_t nb, uint32_t split,
                                                    uint32_t* __restrict__ bcrc) {
  const uint32_t b = blockIdx.x, l = threadIdx.x;
  if (b >= nb) return;
  const uint32_t lo = binst[b], hi = binst[b + 1];
  const uint32_t per = ceil_div(hi - lo, split);
  uint32_t c = 0;
  for (uint32_t w = l; w < split; w += 64) {
    const uint32_t e = min(hi, min(hi, lo + w * per) + per);
    c ^= crc_pow_mul(part[b * split + w], xp2, hi - e);
  }
  if (l == 63) c ^= crc_pow_mul(0xffffffffu, xp2, hi - lo);  // the initial register, shifted through
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) c ^= (uint32_t)__shfl_xor((int)c, o, 64);
  if (l == 0) bcrc[b] = ~c;
}

// In-use bitmap (8 words) per block; blocks are boff[b]..boff[b+1] of blk.  kInUseSplit
// workgroups per block mark seen bytes in LDS flags from 16-byte loads and OR their bitmap
// into the (zeroed) global one; k_ninuse counts.
constexpr uint32_t kInUseSplit = 16;
__global__ void __launch_bounds__(kT) k_in_use(const uint8_t* __restrict__ blk, const uint32_t* __restrict__ boff,
                                               uint32_t* __restrict__ inuse) {
  __shared__ uint8_t seen[256];
  const uint32_t b = blockIdx.y;
  seen[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lo = boff[b], hi = boff[b + 1];
  const uint32_t per = (ceil_div(hi - lo, kInUseSplit) + 15) & ~15u;
  const uint32_t s0 = lo + blockIdx.x * per, s1 = min(hi, s0 + per);
  // head bytes up to 16-byte alignment, aligned 16-byte words, tail bytes
  const uint32_t a0 = min(s1, (s0 + 15) & ~15u), a1 = max(a0, s1 & ~15u);
  for (uint32_t i = s0 + threadIdx.x; i < a0; i += kT) seen[blk[i]] = 1;
  for (uint32_t i = a1 + threadIdx.x; i < s1; i += kT) seen[blk[i]] = 1;
  for (uint32_t i = a0 + threadIdx.x * 16; i < a1; i += kT * 16) {
    const uint4 q = *reinterpret_cast<const uint4*>(blk + i);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 16; k++) seen[(w[k >> 2] >> (8 * (k & 3))) & 0xffu] = 1;
  }
  __syncthreads();
  const uint64_t m = __ballot(seen[threadIdx.x] != 0);
  if (__lane_id() < 2) {
    const uint32_t word = (uint32_t)(m >> (32 * __lane_id()));
    if (word) atomicOr(&inuse[b * 8 + (threadIdx.x >> 6) * 2 + __lane_id()], word);
  }
}

__global__ void k_ninuse(const uint32_t* __restrict__ inuse, uint32_t nb, uint32_t* __restrict__ ninuse) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) c += __builtin_popcount(inuse[b * 8 + k]);
  ninuse[b] = c;
}

// Primitive period of each block: smallest divisor p of n with blk[i] == blk[i+p] for
// all i < n-p (then the block is w^(n/p)); p = n when aperiodic.
__global__ void __launch_bounds__(kT) k_period(const uint8_t* __restrict__ blk, const uint32_t* __restrict__ boff,
                                               uint32_t* __restrict__ period) {
  __shared__ uint32_t divs[512];
  __shared__ uint32_t ndiv;
  __shared__ int bad;
  const int b = blockIdx.x;
  const uint32_t lo = boff[b], n = boff[b + 1] - lo;
  if (threadIdx.x == 0) ndiv = 0;
  __syncthreads();
  for (uint32_t d = 1 + threadIdx.x; (uint64_t)d * d <= n; d += kT) {
    if (n % d == 0) {
      uint32_t k = atomicAdd(&ndiv, 1u);
      if (k < 512) divs[k] = d;
      if (d != n / d) {
        k = atomicAdd(&ndiv, 1u);
        if (k < 512) divs[k] = n / d;
      }
    }
  }
  __syncthreads();
  const uint32_t nd = ndiv < 512 ? ndiv : 512;
  // ascending order (simple rank sort, nd <= 512)
  __shared__ uint32_t sorted[512];
  for (uint32_t i = threadIdx.x; i < nd; i += kT) {
    uint32_t v = divs[i], r = 0;
    for (uint32_t j = 0; j < nd; j++) r += divs[j] < v;
    sorted[r] = v;
  }
  __syncthreads();
  // every divisor is first tested on the block's first 64 positions, all at once (one thread
  // per divisor); only the survivors get the whole-block check, in ascending order.  An
  // aperiodic block (all text) has none but n, so its dozens of divisors no longer cost a
  // chain of whole-workgroup rounds each (a 100 MB call: 370 us of k_period).
  __shared__ uint8_t cand[512];
  for (uint32_t i = threadIdx.x; i < nd; i += kT) {
    const uint32_t p = sorted[i];
    bool ok = p < n;
    const uint32_t m = ok ? min(64u, n - p) : 0u;
    for (uint32_t j = 0; ok && j < m; j += 16) {
      uint4 x, y;
      __builtin_memcpy(&x, blk + lo + j, 16);
      __builtin_memcpy(&y, blk + lo + j + p, 16);
      const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
      for (uint32_t c = 0; c < 16 && j + c < m; c++) ok = ok && (((xs[c >> 2] ^ ys[c >> 2]) >> (8 * (c & 3))) & 0xffu) == 0;
    }
    cand[i] = ok ? 1 : 0;
  }
  __syncthreads();
  uint32_t result = n;
  for (uint32_t q = 0; q < nd; q++) {
    const uint32_t p = sorted[q];
    if (p >= n) break;
    if (!cand[q]) continue;  // (uniform: every thread reads the same flag)
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    // 16 bytes per thread and step (unaligned loads; the block buffer is padded), 64 KB per
    // step: the period that holds reads the whole block (single-byte runs: 900 kB)
    for (uint32_t i0 = 0; i0 < n - p; i0 += kT * 16 * 16) {
      bool diff = false;
#pragma unroll 4
      for (uint32_t k = 0; k < 16; k++) {
        const uint32_t i = i0 + (k * kT + threadIdx.x) * 16;
        if (i >= n - p) break;
        uint4 x, y;
        __builtin_memcpy(&x, blk + lo + i, 16);
        __builtin_memcpy(&y, blk + lo + i + p, 16);
        const uint32_t m = n - p - i;  // bytes of this piece that count
        if (m >= 16) {
          diff |= (x.x != y.x) | (x.y != y.y) | (x.z != y.z) | (x.w != y.w);
        } else {
          const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
          for (uint32_t c = 0; c < m; c++)
            diff |= ((xs[c >> 2] ^ ys[c >> 2]) >> (8 * (c & 3))) & 0xffu;
        }
      }
      if (diff) bad = 1;
      __syncthreads();
      const bool stop = bad;
      __syncthreads();  // every thread has read the flag before the next chunk may set it
      if (stop) break;
    }
    __syncthreads();
    if (!bad) { result = p; break; }
    __syncthreads();
  }
  if (threadIdx.x == 0) period[b] = result;
}

// Quasi-periodic blocks (qsa.h): the smallest period p <= kQsaMaxPeriod, 2p <= n, of a block
// that is not a power of a shorter word, when p does not divide n (else 0).  Thread t tests
// p = t + 1 on the block's first 64 positions; the candidates left are verified in ascending
// order by the whole workgroup (text blocks rarely leave any).
__global__ void __launch_bounds__(kT) k_qperiod(const uint8_t* __restrict__ blk, const uint32_t* __restrict__ boff,
                                                const uint32_t* __restrict__ period, uint32_t* __restrict__ qper) {
  static_assert(kQsaMaxPeriod <= (uint32_t)kT, "one candidate period per thread");
  __shared__ uint64_t cand[kT / 64];
  __shared__ int bad;
  const uint32_t b = blockIdx.x, lo = boff[b], n = boff[b + 1] - lo;
  const uint8_t* t = blk + lo;
  const uint32_t pmax = min(kQsaMaxPeriod, n / 2);
  if (period[b] != n || n < 4) {  // periodic blocks go to A5
    if (threadIdx.x == 0) qper[b] = 0;
    return;
  }
  const uint32_t p = threadIdx.x + 1;
  bool ok = p <= pmax;
  for (uint32_t i = 0; ok && i < min(64u, n - p); i++) ok = t[i] == t[i + p];
  const uint64_t m = __ballot(ok);
  if (__lane_id() == 0) cand[threadIdx.x >> 6] = m;
  __syncthreads();
  uint32_t found = 0;
  for (uint32_t w = 0; w < kT / 64 && !found; w++) {
    uint64_t mw = cand[w];
    while (mw && !found) {
      const uint32_t q = w * 64 + (uint32_t)__builtin_ctzll(mw) + 1;
      mw &= mw - 1;
      if (threadIdx.x == 0) bad = 0;
      __syncthreads();
      for (uint32_t i0 = 0; i0 < n - q; i0 += kT * 16) {
        for (uint32_t i = i0 + threadIdx.x; i < n - q && i < i0 + kT * 16; i += kT)
          if (t[i] != t[i + q]) bad = 1;
        __syncthreads();
        const bool stop = bad;
        __syncthreads();  // every thread has read the flag before the next chunk may set it
        if (stop) break;
      }
      __syncthreads();
      if (!bad) found = q;  // the smallest period of the block
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) qper[b] = (found && n % found != 0) ? found : 0u;
}

}  // namespace

// ------------------------------------------------------------------------------------
void rle1_stage(Workspace& ws, const uint8_t* d_in, uint64_t n, int level, bool final_batch,
                bool tail_merge, Rle1Result& res, hipStream_t st, hipStream_t crc_st, hipEvent_t crc_in,
                hipEvent_t crc_out) {
  const uint32_t nblock_max = 100000u * (uint32_t)level - 19u;
  res.nblocks = 0;
  res.consumed = 0;
  res.m = 0;
  if (n == 0) return;
  const uint64_t tiles = ceil_div64(n, kTile);
  const uint64_t mcap = n + n / 4 + 64;
  uint32_t* tmax = ws.u32("rle_tmax", tiles + 64);
  uint32_t* tsum = ws.u32("rle_tsum", tiles + 64);
  uint32_t* tinfo = ws.u32("rle_tinfo", tiles + 64);
  uint32_t* scratch = ws.u32z("rle_scan", scan_scratch_words(tiles) + 64);
  uint32_t* mtot = ws.u32("rle_m", 16);
  uint8_t* blk = ws.u8("blk", mcap + 64);
  uint32_t* cbits = ws.u32("rle_cbits", mcap / 32 + 64);
  const uint32_t max_blocks = (uint32_t)(mcap / nblock_max + 8);
  uint32_t* boff = ws.u32("boff", max_blocks + 2);
  uint32_t* binst = ws.u32("binst", max_blocks + 2);
  uint32_t* nbl = mtot + 4;

  k_rle_count<<<ceil_div64(tiles, kRleG), kT, 0, st>>>(d_in, n, tiles, tmax, tinfo);
  HIP_OK(hipGetLastError());
  scan_u32(ScanOp::Max, true, tmax, tmax, tiles, nullptr, scratch, st);
  k_rle_fix<<<ceil_div64(tiles, kT), kT, 0, st>>>(tmax, tinfo, tiles, tsum);
  HIP_OK(hipGetLastError());
  scan_u32(ScanOp::Sum, true, tsum, tsum, tiles, mtot, scratch, st);
  HIP_OK(hipMemsetAsync(cbits, 0, (mcap / 32 + 64) * 4, st));
  k_emit<<<ceil_div64(tiles, kRleG), kT, 0, st>>>(d_in, n, tiles, tmax, tsum, blk, cbits, mtot + 8, tinfo);
  HIP_OK(hipGetLastError());
  if (BZG_EMIT_INRUN) {
    k_emit_runs<<<ceil_div64(tiles, kT), kT, 0, st>>>(d_in, n, tiles, tmax, tsum, tinfo, blk, cbits);
    HIP_OK(hipGetLastError());
  }

  // the cut walk of k_segment_fill from fill 0 (cuts into boff[1..]), then boff/nblocks
  k_segment_fill<<<1, 64, 0, st>>>(cbits, mtot, nblock_max, 0u, (final_batch && tail_merge) ? 1 : 0, mtot + 8,
                                   boff + 1, mtot + 12, max_blocks - 1);
  HIP_OK(hipGetLastError());
  k_segment_finish<<<1, 64, 0, st>>>(mtot, mtot + 12, final_batch ? 1 : 0, boff, nbl);
  HIP_OK(hipGetLastError());
  uint32_t hv[2];
  ws.read_small({{hv, mtot, 4}, {hv + 1, nbl, 4}}, st);
  if (hv[1] == 0xffffffffu) throw HipFailure(hipErrorUnknown);
  res.m = hv[0];
  res.nblocks = hv[1];
  // input offsets of the block starts (chunk starts): binst[b] for b < nblocks (+ the
  // incomplete block's start for a non-final batch); binst[nblocks] = n for a final batch
  {
    const uint32_t nq = final_batch ? res.nblocks : res.nblocks + 1;
    if (nq > 0) {
      k_chunk_inpos<<<nq, kT, 0, st>>>(d_in, n, tmax, tsum, (uint32_t)tiles, boff, nq, binst);
      HIP_OK(hipGetLastError());
    }
    if (final_batch) {
      k_set_word<<<1, 64, 0, st>>>(binst + res.nblocks, (uint32_t)n);
      HIP_OK(hipGetLastError());
    }
  }
  if (res.nblocks == 0) {  // non-final batch with no complete block: consume nothing
    res.consumed = final_batch ? n : 0;
    return;
  }
  // binst[nblocks] is n for a final batch, else the input start of the incomplete block
  // that opens the next batch (a chunk start, so RLE1 restarts there with fresh state).
  std::vector<uint32_t> hbi(res.nblocks + 1);
  ws.read_small(hbi.data(), binst, 4ull * (res.nblocks + 1), st);
  res.consumed = final_batch ? n : hbi[res.nblocks];

  const int B = (int)res.nblocks;
  uint32_t* bcrc = ws.u32("bcrc", max_blocks + 2);
  // sub-ranges per block from the largest block input (long runs: a block spans up to 46 MB),
  // so that a batch mixing ordinary blocks with one long-run block still splits the long one
  uint32_t maxin = 0;
  for (int b = 0; b < B; b++) maxin = std::max(maxin, hbi[b + 1] - hbi[b]);
  const uint32_t split = (uint32_t)std::min<uint64_t>(kCrcSplitMax, std::max<uint64_t>(kCrcSplit, ceil_div64(maxin, 1u << 19)));
  uint32_t* cpart = ws.u32("crc_part", (size_t)(B + 2) * split);
  // the block CRCs are read only by the packing: on a side stream they overlap the sort
  const uint32_t* ctab = ws.crc_table();
  const uint32_t* xtab = ws.xpow2_table();
  // every buffer the side stream touches (here and in block_info_stage) is allocated, on st,
  // before crc_in is recorded: the stream-ordered allocator lets crc_st use memory only once it
  // is ordered behind the allocation
  (void)ws.u32("inuse", (size_t)(B + 2) * 8);
  (void)ws.u32("ninuse", B + 2);
  hipStream_t cs = st;
  if (crc_st && crc_in && crc_out) {
    HIP_OK(hipEventRecord(crc_in, st));
    HIP_OK(hipStreamWaitEvent(crc_st, crc_in, 0));
    cs = crc_st;
  }
  k_block_crc<<<dim3(split, B), kT, 0, cs>>>(d_in, binst, ctab, xtab, split, cpart, tinfo, n);
  HIP_OK(hipGetLastError());
  k_crc_combine<<<B, 64, 0, cs>>>(binst, cpart, xtab, B, split, bcrc);
  HIP_OK(hipGetLastError());
  res.bcrc = bcrc;
  res.blk = blk;
  res.boff = boff;
  res.binst = binst;
  block_info_stage(ws, res, st, cs);
  if (cs != st) HIP_OK(hipEventRecord(crc_out, cs));
}

// ---- one region of a sharded stream ------------------------------------
// seg_map_stage: RLE1 chunk map (chunk-start bitmap, output length) of d_in[0, n), a region
// that starts at a chunk start.  seg_walk_stage: the cut walk for a given open-block fill,
// returning region-relative input offsets.  The map is kept in `ws` between the two calls.
void seg_map_stage(Workspace& ws, const uint8_t* d_in, uint64_t n, hipStream_t st) {
  if (n == 0) return;
  const uint64_t tiles = ceil_div64(n, kTile);
  const uint64_t mcap = n + n / 4 + 64;
  uint32_t* tmax = ws.u32("seg_tmax", tiles + 64);
  uint32_t* tsum = ws.u32("seg_tsum", tiles + 64);
  uint32_t* tinfo = ws.u32("seg_tinfo", tiles + 64);
  uint32_t* scratch = ws.u32z("seg_scan", scan_scratch_words(tiles) + 64);
  uint32_t* mtot = ws.u32("seg_m", 16);
  uint32_t* cbits = ws.u32("seg_cbits", mcap / 32 + 64);
  k_rle_count<<<ceil_div64(tiles, kRleG), kT, 0, st>>>(d_in, n, tiles, tmax, tinfo);
  HIP_OK(hipGetLastError());
  scan_u32(ScanOp::Max, true, tmax, tmax, tiles, nullptr, scratch, st);
  k_rle_fix<<<ceil_div64(tiles, kT), kT, 0, st>>>(tmax, tinfo, tiles, tsum);
  HIP_OK(hipGetLastError());
  scan_u32(ScanOp::Sum, true, tsum, tsum, tiles, mtot, scratch, st);
  HIP_OK(hipMemsetAsync(cbits, 0, (mcap / 32 + 64) * 4, st));
  k_emit<<<ceil_div64(tiles, kRleG), kT, 0, st>>>(d_in, n, tiles, tmax, tsum, nullptr, cbits, mtot + 8, tinfo);
  HIP_OK(hipGetLastError());
  if (BZG_EMIT_INRUN) {
    k_emit_runs<<<ceil_div64(tiles, kT), kT, 0, st>>>(d_in, n, tiles, tmax, tsum, tinfo, nullptr, cbits);
    HIP_OK(hipGetLastError());
  }
}

void seg_walk_stage(Workspace& ws, const uint8_t* d_in, uint64_t n, int level, uint32_t fill_in,
                    bool final_region, std::vector<uint64_t>& cuts, uint64_t& last_chunk, uint32_t& last_fill,
                    hipStream_t st) {
  cuts.clear();
  last_chunk = 0;
  last_fill = fill_in;
  if (n == 0) return;
  const uint32_t nblock_max = 100000u * (uint32_t)level - 19u;
  const uint64_t tiles = ceil_div64(n, kTile);
  const uint64_t mcap = n + n / 4 + 64;
  uint32_t* tmax = ws.u32("seg_tmax", tiles + 64);
  uint32_t* tsum = ws.u32("seg_tsum", tiles + 64);
  uint32_t* mtot = ws.u32("seg_m", 16);
  uint32_t* cbits = ws.u32("seg_cbits", mcap / 32 + 64);
  const uint32_t max_cuts = (uint32_t)(mcap / nblock_max + 8);
  uint32_t* qpos = ws.u32("seg_qpos", max_cuts + 2);
  uint32_t* inpos = ws.u32("seg_inpos", max_cuts + 2);
  uint32_t* res = mtot + 12;
  k_segment_fill<<<1, 64, 0, st>>>(cbits, mtot, nblock_max, fill_in, final_region ? 1 : 0, mtot + 8, qpos, res,
                                   max_cuts);
  HIP_OK(hipGetLastError());
  uint32_t hres[3];
  HIP_OK(hipMemcpyAsync(hres, res, 12, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  if (hres[0] == 0xffffffffu) throw HipFailure(hipErrorUnknown);
  const uint32_t nq = hres[0] + 1;
  k_chunk_inpos<<<nq, kT, 0, st>>>(d_in, n, tmax, tsum, (uint32_t)tiles, qpos, nq, inpos);
  HIP_OK(hipGetLastError());
  std::vector<uint32_t> h(nq);
  HIP_OK(hipMemcpyAsync(h.data(), inpos, 4ull * nq, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  for (uint32_t i = 0; i + 1 < nq; i++) cuts.push_back(h[i]);
  last_chunk = h[nq - 1];
  last_fill = hres[2];
}

void block_info_stage(Workspace& ws, Rle1Result& res, hipStream_t st, hipStream_t side) {
  const uint32_t B = res.nblocks;
  if (B == 0) return;
  res.inuse = ws.u32("inuse", (size_t)(B + 2) * 8);
  res.ninuse = ws.u32("ninuse", B + 2);
  res.period = ws.u32("period", B + 2);
  // in-use maps: read by MTF and the tables, not the sort (side: rle1_stage's CRC stream)
  hipStream_t iu = side ? side : st;
  HIP_OK(hipMemsetAsync(res.inuse, 0, (size_t)B * 8 * 4, iu));
  k_in_use<<<dim3(kInUseSplit, B), kT, 0, iu>>>(res.blk, res.boff, res.inuse);
  HIP_OK(hipGetLastError());
  k_ninuse<<<ceil_div(B, kT), kT, 0, iu>>>(res.inuse, B, res.ninuse);
  HIP_OK(hipGetLastError());
  k_period<<<B, kT, 0, st>>>(res.blk, res.boff, res.period);
  HIP_OK(hipGetLastError());
  res.qper = ws.u32("qper", B + 2);
  k_qperiod<<<B, kT, 0, st>>>(res.blk, res.boff, res.period, res.qper);
  HIP_OK(hipGetLastError());
  copyrank_count_stage(res, ws, st);
}

}  // namespace bzg
