// scan.hip -- device-wide u32 scans.  Tile = 256 threads x 16 elements (4096).  One tile: one
// workgroup.  Up to 64 tiles: one launch, a single pass with decoupled look-back (each tile
// publishes its aggregate, then its inclusive prefix, in a 64-bit flag word; a tile's first
// wave reads the words of all the tiles before it at once).  More: reduce, scan of the
// aggregates, apply.
// Tiles take their index from a ticket counter in the order they start, so a tile only waits
// for tiles already running.  The last tile to finish clears the flags and counters for the
// next scan on the same scratch (which must be zero when first used: Workspace::u32z).
#include "scan.h"

namespace bzg {

namespace {
constexpr int kThreads = 256;
constexpr int kPer = 16;
constexpr int kTile = kThreads * kPer;

template <ScanOp OP>
__device__ __forceinline__ uint32_t comb(uint32_t a, uint32_t b) {
  if constexpr (OP == ScanOp::Sum) return a + b;
  else return a > b ? a : b;
}

template <ScanOp OP>
__global__ void __launch_bounds__(kThreads) k_tile_reduce(const uint32_t* __restrict__ in, size_t n,
                                                          uint32_t* __restrict__ agg) {
  __shared__ uint32_t sh[kThreads / 64];
  const size_t base = (size_t)blockIdx.x * kTile;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    size_t i = base + (size_t)k * kThreads + threadIdx.x;
    if (i < n) acc = comb<OP>(acc, in[i]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc = comb<OP>(acc, (uint32_t)__shfl_xor((int)acc, o, 64));
  if (__lane_id() == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kThreads / 64; w++) t = comb<OP>(t, sh[w]);
    agg[blockIdx.x] = t;
  }
}

// Scans one tile in place given a carry-in (exclusive or inclusive).
template <ScanOp OP>
__global__ void __launch_bounds__(kThreads) k_tile_scan(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                        size_t n, const uint32_t* __restrict__ carry,
                                                        int exclusive, uint32_t* __restrict__ total) {
  __shared__ uint32_t sh[kThreads / 64];
  const size_t base = (size_t)blockIdx.x * kTile + (size_t)threadIdx.x * kPer;
  uint32_t v[kPer];
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    size_t i = base + k;
    v[k] = i < n ? in[i] : 0u;
    acc = comb<OP>(acc, v[k]);
  }
  // block inclusive scan of per-thread aggregates
  uint32_t x = acc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = (uint32_t)__shfl_up((int)x, o, 64);
    if (__lane_id() >= o) x = comb<OP>(x, t);
  }
  if (__lane_id() == 63) sh[threadIdx.x >> 6] = x;
  __syncthreads();
  uint32_t pre = carry ? carry[blockIdx.x] : 0u;
  for (int w = 0; w < (int)(threadIdx.x >> 6); w++) pre = comb<OP>(pre, sh[w]);
  // exclusive prefix of this thread
  uint32_t run = comb<OP>(pre, x);  // inclusive through this thread
  uint32_t ex = (uint32_t)__shfl_up((int)x, 1, 64);
  uint32_t cur = (__lane_id() == 0) ? pre : comb<OP>(pre, ex);
  (void)run;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    size_t i = base + k;
    uint32_t nxt = comb<OP>(cur, v[k]);
    if (i < n) out[i] = exclusive ? cur : nxt;
    cur = nxt;
  }
  if (total && blockIdx.x == gridDim.x - 1 && threadIdx.x == kThreads - 1) *total = cur;
}

// flag word of a tile: status << 32 | value (status 0: nothing yet, 1: aggregate, 2: inclusive)
__device__ __forceinline__ uint64_t flag_load(const uint64_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void flag_store(uint64_t* f, uint32_t status, uint32_t v) {
  __hip_atomic_store(f, ((uint64_t)status << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// state[0]: ticket, state[1]: finished tiles; flags[0, tiles)
template <ScanOp OP>
__global__ void __launch_bounds__(kThreads) k_scan_1p(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                      size_t n, int exclusive, uint32_t* __restrict__ total,
                                                      uint32_t* __restrict__ state, uint64_t* __restrict__ flags,
                                                      uint32_t tiles) {
  __shared__ uint32_t sh[kThreads / 64];
  __shared__ uint32_t s_tile, s_pre;
  if (threadIdx.x == 0) s_tile = atomicAdd(&state[0], 1u);
  __syncthreads();
  const uint32_t t = s_tile;
  const size_t base = (size_t)t * kTile + (size_t)threadIdx.x * kPer;
  uint32_t v[kPer];
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const size_t i = base + k;
    v[k] = i < n ? in[i] : 0u;
    acc = comb<OP>(acc, v[k]);
  }
  uint32_t x = acc;  // inclusive over the wave's threads
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
    if (__lane_id() >= o) x = comb<OP>(x, y);
  }
  if (__lane_id() == 63) sh[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x < 64) {  // the first wave publishes the aggregate and looks back
    uint32_t agg = 0;
    for (int w = 0; w < kThreads / 64; w++) agg = comb<OP>(agg, sh[w]);
    uint32_t pre = 0;
    if (t == 0) {
      if (threadIdx.x == 0) flag_store(&flags[0], 2u, agg);
    } else {
      if (threadIdx.x == 0) flag_store(&flags[t], 1u, agg);
      // tiles t - 1 - lane, 64 at a time, until one of them holds an inclusive prefix
      for (int64_t j = (int64_t)t - 1;; j -= 64) {
        const int64_t q = j - (int64_t)__lane_id();
        uint64_t f = q >= 0 ? flag_load(&flags[q]) : (2ull << 32);
        while (__ballot((f >> 32) == 0) != 0) {
          if ((f >> 32) == 0) f = flag_load(&flags[q]);
        }
        const uint64_t incl = __ballot((f >> 32) == 2);
        // lanes up to the first inclusive one (the nearest tile) contribute
        const uint32_t stop = incl ? (uint32_t)__builtin_ctzll(incl) : 63u;
        uint32_t c = __lane_id() <= stop ? (uint32_t)f : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c = comb<OP>(c, (uint32_t)__shfl_xor((int)c, o, 64));
        pre = comb<OP>(pre, c);
        if (incl) break;
      }
      if (threadIdx.x == 0) flag_store(&flags[t], 2u, comb<OP>(pre, agg));
    }
    if (threadIdx.x == 0) s_pre = pre;
  }
  __syncthreads();
  uint32_t pre = s_pre;
  for (int w = 0; w < (int)(threadIdx.x >> 6); w++) pre = comb<OP>(pre, sh[w]);
  const uint32_t ex = (uint32_t)__shfl_up((int)x, 1, 64);
  uint32_t cur = (__lane_id() == 0) ? pre : comb<OP>(pre, ex);
#pragma unroll
  for (int k = 0; k < kPer; k++) {
    const size_t i = base + k;
    const uint32_t nxt = comb<OP>(cur, v[k]);
    if (i < n) out[i] = exclusive ? cur : nxt;
    cur = nxt;
  }
  if (total && t == tiles - 1 && threadIdx.x == kThreads - 1) *total = cur;
  // the last tile to finish (every look-back is over) resets the scratch for the next scan;
  // the fences order each tile's flag stores before its count, and the count before the reset
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    s_tile = atomicAdd(&state[1], 1u);
    __threadfence();
  }
  __syncthreads();
  if (s_tile == tiles - 1) {
    for (uint32_t i = threadIdx.x; i < tiles; i += kThreads) flags[i] = 0;
    if (threadIdx.x == 0) {
      state[0] = 0;
      state[1] = 0;
    }
  }
}

}  // namespace

// Single pass up to this many tiles (one look-back round reaches tile 0); above it the
// look-back chains and its spinning waves cost more than the two extra launches of the
// reduce / scan-of-aggregates / apply passes (text at 1 GB: BWT +1.9 ms, long repeats +6.8 ms
// with a single pass at every size).
constexpr size_t kOnePassTiles = 64;
constexpr size_t kStateWords = 16 + 2 * kOnePassTiles;  // ticket, finished count; 64-bit flags

size_t scan_scratch_words(size_t n) {
  size_t words = 0;
  while (n > (size_t)kTile) {
    n = ceil_div64(n, kTile);
    words += n + 64;
  }
  return kStateWords + words + 64;
}

// reduce, scan of the aggregates (recursively), apply; `scratch` past the one-pass state
static void scan_passes(ScanOp op, bool exclusive, const uint32_t* in, uint32_t* out, size_t n, uint32_t* total,
                        uint32_t* scratch, hipStream_t st) {
  const size_t tiles = ceil_div64(n, kTile);
  if (tiles == 1) {
    if (op == ScanOp::Sum)
      k_tile_scan<ScanOp::Sum><<<1, kThreads, 0, st>>>(in, out, n, nullptr, exclusive, total);
    else
      k_tile_scan<ScanOp::Max><<<1, kThreads, 0, st>>>(in, out, n, nullptr, exclusive, total);
    HIP_OK(hipGetLastError());
    return;
  }
  uint32_t* agg = scratch;
  uint32_t* rest = scratch + tiles + 64;
  if (op == ScanOp::Sum)
    k_tile_reduce<ScanOp::Sum><<<tiles, kThreads, 0, st>>>(in, n, agg);
  else
    k_tile_reduce<ScanOp::Max><<<tiles, kThreads, 0, st>>>(in, n, agg);
  HIP_OK(hipGetLastError());
  scan_passes(op, true, agg, agg, tiles, nullptr, rest, st);
  if (op == ScanOp::Sum)
    k_tile_scan<ScanOp::Sum><<<tiles, kThreads, 0, st>>>(in, out, n, agg, exclusive, total);
  else
    k_tile_scan<ScanOp::Max><<<tiles, kThreads, 0, st>>>(in, out, n, agg, exclusive, total);
  HIP_OK(hipGetLastError());
}

void scan_u32(ScanOp op, bool exclusive, const uint32_t* in, uint32_t* out, size_t n,
              uint32_t* total, uint32_t* scratch, hipStream_t st) {
  if (n == 0) {
    if (total) HIP_OK(hipMemsetAsync(total, 0, 4, st));
    return;
  }
  const size_t tiles = ceil_div64(n, kTile);
  if (tiles == 1) {
    if (op == ScanOp::Sum)
      k_tile_scan<ScanOp::Sum><<<1, kThreads, 0, st>>>(in, out, n, nullptr, exclusive, total);
    else
      k_tile_scan<ScanOp::Max><<<1, kThreads, 0, st>>>(in, out, n, nullptr, exclusive, total);
    HIP_OK(hipGetLastError());
    return;
  }
  static const size_t one_pass = (size_t)std::min<long long>((long long)kOnePassTiles, env_ll("BZG_SCAN_1P", (long long)kOnePassTiles));
  if (tiles > one_pass) {
    scan_passes(op, exclusive, in, out, n, total, scratch + kStateWords, st);
    return;
  }
  uint32_t* state = scratch;
  uint64_t* flags = reinterpret_cast<uint64_t*>(scratch + 16);
  if (op == ScanOp::Sum)
    k_scan_1p<ScanOp::Sum><<<tiles, kThreads, 0, st>>>(in, out, n, exclusive, total, state, flags, (uint32_t)tiles);
  else
    k_scan_1p<ScanOp::Max><<<tiles, kThreads, 0, st>>>(in, out, n, exclusive, total, state, flags, (uint32_t)tiles);
  HIP_OK(hipGetLastError());
}

}  // namespace bzg
