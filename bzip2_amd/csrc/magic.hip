// magic.hip -- block-boundary discovery in an existing .bz2 stream.
//
// Reference behaviour restated (bzip2recover.c:360-395): the stream is read bit by bit into a
// 64-bit shift register; every bit position where the last 48 bits equal the block-header
// magic 0x314159265359 (bzip2recover.c:284-285) or the end-of-stream magic 0x177245385090
// (287-288) is a boundary.  Blocks are not byte-aligned, so a magic can start at any bit.
//
// Data-parallel form: a magic starting at bit 8p + k (k = 0..7) lies in bytes p..p+6.  A thread
// takes 16 start bytes at a time (with 8 bytes of look-ahead, one 16-byte and one 8-byte load);
// a byte-pair filter (below) rejects almost every position, and survivors compare the 48-bit
// field at all 8 shifts of the big-endian 64-bit window of bytes p..p+7.  Matches go to an
// unordered list (atomic counter; boundaries are about one per 100-900 kB) that the host sorts.
// The scan is HBM-bound: 1 byte read per byte of stream.
#include <algorithm>
#include <vector>

#include "common.h"

namespace bzg {
namespace {
constexpr uint64_t kMagicBlock = 0x314159265359ull;
constexpr uint64_t kMagicEos = 0x177245385090ull;
constexpr int kT = 256;
// Filter: bytes p+1, p+2 of a match are fixed by the magic and the shift k, so the 16
// possible byte pairs go into a 65536-bit LDS table (built once per workgroup; the grid
// strides over the stream) and one LDS lookup rejects a position with probability
// 1 - 16/65536.  Few waves ever take the compare path, so it costs no divergence.
constexpr int kGrid = 2048;  // 8 workgroups per CU

__global__ void __launch_bounds__(kT) k_find_magics(const uint8_t* __restrict__ x, uint64_t n,
                                                    unsigned long long* __restrict__ out, uint64_t cap,
                                                    unsigned long long* __restrict__ cnt) {
  __shared__ uint32_t tab[2048];
  for (int i = threadIdx.x; i < 2048; i += kT) tab[i] = 0;
  __syncthreads();
  if (threadIdx.x < 16) {
    const uint64_t mg = threadIdx.x < 8 ? kMagicBlock : kMagicEos;
    const int k = threadIdx.x & 7;
    const uint32_t pair = (uint32_t)(((mg >> (32 + k)) & 0xff) << 8 | ((mg >> (24 + k)) & 0xff));
    atomicOr(&tab[pair >> 5], 1u << (pair & 31));
  }
  __syncthreads();
  const uint64_t nbits = 8 * n;
  const bool aligned = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  for (uint64_t c = (uint64_t)blockIdx.x * kT + threadIdx.x; c * 16 < n; c += (uint64_t)gridDim.x * kT) {
    const uint64_t base = c * 16;
    uint32_t w[6];  // bytes base..base+23, big-endian words (byte 4q is the top byte of w[q])
    if (base + 24 <= n && aligned) {
      const uint4 a = *reinterpret_cast<const uint4*>(x + base);
      const uint2 d = *reinterpret_cast<const uint2*>(x + base + 16);
      w[0] = __builtin_bswap32(a.x);
      w[1] = __builtin_bswap32(a.y);
      w[2] = __builtin_bswap32(a.z);
      w[3] = __builtin_bswap32(a.w);
      w[4] = __builtin_bswap32(d.x);
      w[5] = __builtin_bswap32(d.y);
    } else {
#pragma unroll
      for (int q = 0; q < 6; q++) {
        uint32_t v = 0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const uint64_t i = base + 4 * q + r;
          v = (v << 8) | (i < n ? x[i] : 0u);
        }
        w[q] = v;
      }
    }
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t b1 = (w[(j + 1) >> 2] >> (24 - 8 * ((j + 1) & 3))) & 0xffu;
      const uint32_t b2 = (w[(j + 2) >> 2] >> (24 - 8 * ((j + 2) & 3))) & 0xffu;
      const uint32_t pair = b1 << 8 | b2;
      if (!((tab[pair >> 5] >> (pair & 31)) & 1u)) continue;
      // 64-bit window of bytes base+j .. base+j+7
      const int q = j >> 2, r = j & 3;
      const uint64_t hi = ((uint64_t)w[q] << 32) | w[q + 1];
      const uint64_t lo = w[q + 2];
      const uint64_t win = r ? ((hi << (8 * r)) | (lo >> (32 - 8 * r))) : hi;
      const uint64_t pos = base + j;
      for (int k = 0; k < 8; k++) {
        const uint64_t v = (win >> (16 - k)) & 0xffffffffffffull;
        if ((v == kMagicBlock || v == kMagicEos) && 8 * pos + k + 48 <= nbits) {
          const unsigned long long idx = atomicAdd(cnt, 1ull);
          if (idx < cap) out[idx] = ((8 * pos + k) << 1) | (v == kMagicEos ? 1ull : 0ull);
        }
      }
    }
  }
}
}  // namespace

// All magics of d_in[0, n), sorted; returns the number found (out holds min(found, cap)).
uint64_t find_magics_stage(const uint8_t* d_in, uint64_t n, std::vector<uint64_t>& found, hipStream_t st) {
  found.clear();
  if (n == 0) return 0;
  uint64_t cap = n / 4096 + 1024;  // grows and reruns if a stream holds more
  for (;;) {
    unsigned long long* d_out = nullptr;
    unsigned long long* d_cnt = nullptr;
    HIP_OK(hipMallocAsync((void**)&d_out, cap * 8, st));
    HIP_OK(hipMallocAsync((void**)&d_cnt, 8, st));
    HIP_OK(hipMemsetAsync(d_cnt, 0, 8, st));
    const uint64_t wgs = ((n + 15) / 16 + kT - 1) / kT;
    k_find_magics<<<(unsigned)(wgs < kGrid ? wgs : kGrid), kT, 0, st>>>(d_in, n, d_out, cap, d_cnt);
    HIP_OK(hipGetLastError());
    unsigned long long h_cnt = 0;
    HIP_OK(hipMemcpyAsync(&h_cnt, d_cnt, 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (h_cnt <= cap) {
      found.resize(h_cnt);
      if (h_cnt) HIP_OK(hipMemcpyAsync(found.data(), d_out, h_cnt * 8, hipMemcpyDeviceToHost, st));
    }
    HIP_OK(hipFreeAsync(d_out, st));
    HIP_OK(hipFreeAsync(d_cnt, st));
    HIP_OK(hipStreamSynchronize(st));
    if (h_cnt <= cap) break;
    cap = h_cnt;
  }
  std::sort(found.begin(), found.end());
  return found.size();
}

}  // namespace bzg
