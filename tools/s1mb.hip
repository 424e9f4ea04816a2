// Microbenchmark of the S1 scatter pass shapes (development tool, not part of the product):
// one MSD byte pass over n text positions (identity order), tiles of 4096, 256 threads.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint32_t kT = 256, kPerT = 16, kTile = kT * kPerT;

__global__ void __launch_bounds__(kT) k_hist(const uint8_t* __restrict__ text, uint32_t n, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const uint32_t t = blockIdx.x, lo = t * kTile;
  h[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t i = 0; i < kPerT; i++) {
    const uint32_t e = lo + i * kT + threadIdx.x;
    if (e < n) atomicAdd(&h[text[e]], 1u);
  }
  __syncthreads();
  hist[(size_t)t * 256 + threadIdx.x] = h[threadIdx.x];
}

// per-group column scan (groups of kGT tiles): off[t][d] = global base of digit d in tile t
constexpr uint32_t kGT = 220;
__global__ void k_gscan(uint32_t* __restrict__ hist, uint32_t nt) {
  __shared__ uint32_t sh[256];
  const uint32_t g = blockIdx.x, d = threadIdx.x;
  const uint32_t t0 = g * kGT, t1 = min(nt, t0 + kGT);
  uint32_t tot = 0;
  for (uint32_t t = t0; t < t1; t++) tot += hist[(size_t)t * 256 + d];
  sh[d] = tot;
  __syncthreads();
  uint32_t ex = 0;
  for (uint32_t e = 0; e < d; e++) ex += sh[e];
  uint32_t run = t0 * kTile + ex;
  for (uint32_t t = t0; t < t1; t++) {
    const uint32_t c = hist[(size_t)t * 256 + d];
    hist[(size_t)t * 256 + d] = run;
    run += c;
  }
}

__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
  const uint32_t per = n / 8, rem = n % 8, x = b % 8, k = b / 8;
  return x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
}

// column scan: off[t][d] = global base of digit d in tile t
__global__ void k_colscan(uint32_t* __restrict__ hist, uint32_t nt, const uint32_t* __restrict__ dbase) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= 256) return;
  uint32_t run = dbase[d];
  for (uint32_t t = 0; t < nt; t++) {
    const uint32_t c = hist[(size_t)t * 256 + d];
    hist[(size_t)t * 256 + d] = run;
    run += c;
  }
}

__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) {
  uint32_t x;
  __builtin_memcpy(&x, p, 4);
  return x;
}

// V: bit0 = dword key loads (else byte), bit1 = also store the key array, bit2 = LDS staging,
//    bit3 = skip stores entirely, bit4 = non-returning atomics only (hist shape)
__device__ uint32_t g_TP[1200];
__device__ uint32_t g_G[1200 * 4];

template <int V>
__global__ void __launch_bounds__(kT) k_scatter(const uint8_t* __restrict__ text, uint32_t n, const uint32_t* __restrict__ off,
                                                uint32_t* __restrict__ dst, uint32_t* __restrict__ dstk) {
  if (V & 64) {  // prologue chain of the real kernel: binary search of the tile's group + 2 loads
    const uint32_t tt = (V & 32) ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    uint32_t lo_ = 0, hi_ = 1110;
    while (hi_ - lo_ > 1) {
      const uint32_t mid = (lo_ + hi_) >> 1;
      if (g_TP[mid] <= tt) lo_ = mid;
      else hi_ = mid;
    }
    const uint32_t u = g_G[lo_ * 4 + 2];
    if (g_G[u * 4 + 3] == 12345u && threadIdx.x == 999) dst[0] = 0;  // keeps the chain
  }
  __shared__ uint32_t cnt[256], base[256];
  __shared__ uint32_t sh[4];
  __shared__ uint32_t Lv[(V & 4) ? kTile : 1], Lk[(V & 4) ? kTile : 1];
  const uint32_t t = (V & 32) ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x, lo = t * kTile, hi = min(n, lo + kTile);
  const uint32_t d = threadIdx.x;
  cnt[d] = 0;
  const uint32_t gbase = off[(size_t)t * 256 + d];
  base[d] = gbase;
  uint32_t kk[kPerT];
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++) {
    const uint32_t x = min(lo + i * kT + threadIdx.x, n - 1);
    kk[i] = (V & 1) ? __builtin_bswap32(ld_u32(text + x)) : ((uint32_t)text[x] << 24);
  }
  __syncthreads();
  if (V & 16) {
#pragma unroll
    for (int i = 0; i < (int)kPerT; i++)
      if (lo + i * kT + threadIdx.x < hi) atomicAdd(&cnt[kk[i] >> 24], 1u);
    __syncthreads();
    dst[(size_t)t * 256 + d] = cnt[d];
    return;
  }
  uint32_t rk[kPerT];
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++)
    if (lo + i * kT + threadIdx.x < hi) rk[i] = atomicAdd(&cnt[kk[i] >> 24], 1u);
  if (!(V & 4)) {
#pragma unroll
    for (int i = 0; i < (int)kPerT; i++) {
      const uint32_t e = lo + i * kT + threadIdx.x;
      if (e < hi && !(V & 8)) {
        const uint32_t p = base[kk[i] >> 24] + rk[i];
        dst[p] = e;
        if (V & 2) dstk[p] = kk[i] << 8;
      }
    }
    return;
  }
  __syncthreads();
  {
    const uint32_t c = cnt[d];
    // exclusive scan over 256 digits
    uint32_t x = c;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if ((d & 63) >= (uint32_t)o) x += y;
    }
    if ((d & 63) == 63) sh[d >> 6] = x;
    __syncthreads();
    for (uint32_t w = 0; w < (d >> 6); w++) x += sh[w];
    const uint32_t ls = x - c;
    cnt[d] = ls;
    base[d] = gbase - ls;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++) {
    const uint32_t e = lo + i * kT + threadIdx.x;
    if (e < hi) {
      const uint32_t lp = cnt[kk[i] >> 24] + rk[i];
      Lv[lp] = e;
      Lk[lp] = kk[i];
    }
  }
  __syncthreads();
  const uint32_t m = hi - lo;
#pragma unroll
  for (int i = 0; i < (int)kPerT; i++) {
    const uint32_t x = i * kT + threadIdx.x;
    if (x < m && !(V & 8)) {
      const uint32_t k = Lk[x];
      const uint32_t p = base[k >> 24] + x;
      dst[p] = Lv[x];
      if (V & 2) dstk[p] = k << 8;
    }
  }
}

template <int V>
static float run(const uint8_t* text, uint32_t n, const uint32_t* off, uint32_t* dst, uint32_t* dstk) {
  const uint32_t nt = (n + kTile - 1) / kTile;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_scatter<V><<<nt, kT>>>(text, n, off, dst, dstk);
  hipEventRecord(a);
  for (int r = 0; r < 5; r++) k_scatter<V><<<nt, kT>>>(text, n, off, dst, dstk);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

extern "C" int s1mb(const uint8_t* host_text, uint32_t n) {
  const uint32_t nt = (n + kTile - 1) / kTile;
  uint8_t* text;
  uint32_t *hist, *dst, *dstk, *dbase;
  hipMalloc(&text, n + 16);
  hipMalloc(&hist, (size_t)nt * 256 * 4);
  hipMalloc(&dst, (size_t)n * 4 + 64);
  hipMalloc(&dstk, (size_t)n * 4 + 64);
  hipMalloc(&dbase, 256 * 4);
  hipMemcpy(text, host_text, n, hipMemcpyHostToDevice);
  hipMemset(text + n, 0, 16);
  uint32_t cnt[256] = {0}, db[256];
  for (uint32_t i = 0; i < n; i++) cnt[host_text[i]]++;
  uint32_t run_ = 0;
  for (int d = 0; d < 256; d++) { db[d] = run_; run_ += cnt[d]; }
  hipMemcpy(dbase, db, sizeof(db), hipMemcpyHostToDevice);
  k_hist<<<nt, kT>>>(text, n, hist);
  k_colscan<<<1, 256>>>(hist, nt, dbase);
  hipDeviceSynchronize();
  printf("n=%u tiles=%u  one group\n", n, nt);
  printf("V0  byte, rtn atomics, scattered sa          %.3f ms\n", run<0>(text, n, hist, dst, dstk));
  printf("V2  byte + scattered sk                      %.3f ms\n", run<2>(text, n, hist, dst, dstk));
  printf("V4  byte, staged sa                          %.3f ms\n", run<4>(text, n, hist, dst, dstk));
  printf("V6  byte, staged sa+sk                       %.3f ms\n", run<6>(text, n, hist, dst, dstk));
  printf("V32 remap byte, rtn atomics, scattered sa    %.3f ms\n", run<32>(text, n, hist, dst, dstk));
  printf("V34 remap byte + scattered sk                %.3f ms\n", run<34>(text, n, hist, dst, dstk));
  printf("V36 remap byte, staged sa                    %.3f ms\n", run<36>(text, n, hist, dst, dstk));
  printf("V38 remap byte, staged sa+sk                 %.3f ms\n", run<38>(text, n, hist, dst, dstk));
  k_hist<<<nt, kT>>>(text, n, hist);
  k_gscan<<<(nt + kGT - 1) / kGT, 256>>>(hist, nt);
  hipDeviceSynchronize();
  printf("groups of %u tiles\n", kGT);
  printf("V0  byte, rtn atomics, scattered sa          %.3f ms\n", run<0>(text, n, hist, dst, dstk));
  printf("V2  byte + scattered sk                      %.3f ms\n", run<2>(text, n, hist, dst, dstk));
  printf("V4  byte, staged sa                          %.3f ms\n", run<4>(text, n, hist, dst, dstk));
  printf("V6  byte, staged sa+sk                       %.3f ms\n", run<6>(text, n, hist, dst, dstk));
  printf("V32 remap byte, rtn atomics, scattered sa    %.3f ms\n", run<32>(text, n, hist, dst, dstk));
  printf("V34 remap byte + scattered sk                %.3f ms\n", run<34>(text, n, hist, dst, dstk));
  printf("V36 remap byte, staged sa                    %.3f ms\n", run<36>(text, n, hist, dst, dstk));
  printf("V38 remap byte, staged sa+sk                 %.3f ms\n", run<38>(text, n, hist, dst, dstk));
  {
    uint32_t tp[1200], gg[1200 * 4] = {0};
    for (int i = 0; i < 1200; i++) tp[i] = i * kGT;
    hipMemcpyToSymbol(HIP_SYMBOL(g_TP), tp, sizeof(tp));
    hipMemcpyToSymbol(HIP_SYMBOL(g_G), gg, sizeof(gg));
    printf("V100 chain remap byte, staged sa             %.3f ms\n", run<100>(text, n, hist, dst, dstk));
    printf("V102 chain remap byte, staged sa+sk          %.3f ms\n", run<102>(text, n, hist, dst, dstk));
    printf("V96  chain remap byte, scattered sa          %.3f ms\n", run<96>(text, n, hist, dst, dstk));
  }
  hipError_t e = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(e));
  hipFree(text); hipFree(hist); hipFree(dst); hipFree(dstk); hipFree(dbase);
  return 0;
}
