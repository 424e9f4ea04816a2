// scan.hip -- device-wide u32 scans.  Tile = 256 threads x 16 elements (4096); each level
// reduces tiles to one aggregate, scans the aggregates (recursively), and applies them.
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
  // wave reduce
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

}  // namespace

size_t scan_scratch_words(size_t n) {
  size_t words = 0;
  while (n > (size_t)kTile) {
    n = ceil_div64(n, kTile);
    words += n + 64;
  }
  return words + 64;
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
  uint32_t* agg = scratch;
  uint32_t* rest = scratch + tiles + 64;
  if (op == ScanOp::Sum)
    k_tile_reduce<ScanOp::Sum><<<tiles, kThreads, 0, st>>>(in, n, agg);
  else
    k_tile_reduce<ScanOp::Max><<<tiles, kThreads, 0, st>>>(in, n, agg);
  HIP_OK(hipGetLastError());
  // exclusive scan of aggregates -> carries
  scan_u32(op, true, agg, agg, tiles, nullptr, rest, st);
  if (op == ScanOp::Sum)
    k_tile_scan<ScanOp::Sum><<<tiles, kThreads, 0, st>>>(in, out, n, agg, exclusive, total);
  else
    k_tile_scan<ScanOp::Max><<<tiles, kThreads, 0, st>>>(in, out, n, agg, exclusive, total);
  HIP_OK(hipGetLastError());
}

}  // namespace bzg
