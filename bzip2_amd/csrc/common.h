// common.h -- shared definitions for the MI355X bzip2 compression engine.
//
// Everything here is gfx950-only HIP: 64-lane wavefronts, 256-thread workgroups by default.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define BZG_WAVE 64

// A wave's SGPR allocation decides how many waves a SIMD admits: 800 / (ceil(sgprs / 16) * 16 +
// 16) (MI355X_MICROARCH.md, residency), so kernels above 80 SGPRs lose the eighth wave per SIMD
// although the compiler's occupancy figure says 8.  Latency-bound kernels cap theirs at 80.
#ifndef BZG_SGPR_CAP
#define BZG_SGPR_CAP 80
#endif
#if BZG_SGPR_CAP > 0
#define BZG_SGPR_LIMIT __attribute__((amdgpu_num_sgpr(BZG_SGPR_CAP)))
#else
#define BZG_SGPR_LIMIT
#endif

#define HIP_OK(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "bzip2_amd: HIP error %s at %s:%d: %s\n", hipGetErrorString(e_),  \
              __FILE__, __LINE__, #expr);                                               \
      throw bzg::HipFailure(e_);                                                        \
    }                                                                                   \
  } while (0)

namespace bzg {

struct HipFailure {
  hipError_t err;
  explicit HipFailure(hipError_t e) : err(e) {}
};
// The caller's output buffer cannot hold the coded stream (BZ_OUTBUFF_FULL); distinct from a
// device allocation failure (HipFailure(hipErrorOutOfMemory) -> BZ_MEM_ERROR).
struct OutBuffFull {};

// Format constants (reference bzlib_private.h:139-152).
constexpr int kMaxAlpha = 258;
constexpr int kMaxCodeLen = 17;
constexpr int kNGroups = 6;
constexpr int kGroupSize = 50;
constexpr int kIters = 4;
constexpr int kMaxSelectors = 2 + 900000 / kGroupSize;  // 18002

// A tuning knob from the environment (host side; read once by the caller's static).
inline long long env_ll(const char* name, long long dflt) {
  const char* e = getenv(name);
  return e && *e ? atoll(e) : dflt;
}

__host__ __device__ inline uint32_t ceil_div(uint32_t a, uint32_t b) { return (a + b - 1) / b; }
__host__ __device__ inline uint64_t ceil_div64(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// ----------------------------------------------------------------------------------------
// Wave-level helpers (64 lanes).
__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int l = __lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T t = __shfl_up(v, o, 64);
    if (__lane_id() >= o) v += t;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_incl_max(T v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T t = __shfl_up(v, o, 64);
    if (__lane_id() >= o) v = v > t ? v : t;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide inclusive sum over blockDim.x threads (multiple of 64, <= 1024).  `sh` needs
// blockDim.x/64 entries.  Returns the inclusive prefix; *total gets the block total.
template <typename T>
__device__ __forceinline__ T block_incl_sum(T v, T* sh, T* total) {
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  T x = wave_incl_sum(v);
  if (__lane_id() == 63) sh[w] = x;
  __syncthreads();
  if (w == 0) {
    T s = (__lane_id() < nw) ? sh[__lane_id()] : T(0);
    s = wave_incl_sum(s);
    if (__lane_id() < nw) sh[__lane_id()] = s;
  }
  __syncthreads();
  T pre = (w > 0) ? sh[w - 1] : T(0);
  if (total) *total = sh[nw - 1];
  __syncthreads();
  return x + pre;
}

template <typename T>
__device__ __forceinline__ T block_incl_max(T v, T* sh) {
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  T x = wave_incl_max(v);
  if (__lane_id() == 63) sh[w] = x;
  __syncthreads();
  if (w == 0) {
    T s = (__lane_id() < nw) ? sh[__lane_id()] : T(0);
    s = wave_incl_max(s);
    if (__lane_id() < nw) sh[__lane_id()] = s;
  }
  __syncthreads();
  T pre = (w > 0) ? sh[w - 1] : T(0);
  __syncthreads();
  return x > pre ? x : pre;
}

// Workgroups are dispatched round-robin over the 8 XCDs (each with its own L2).  Map the
// hardware workgroup index to a logical one so that every XCD walks a contiguous logical
// range: neighbouring data stays in one L2.
constexpr uint32_t kNumXcd = 8;
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nwg) {
  const uint32_t per = nwg / kNumXcd, rem = nwg % kNumXcd;
  const uint32_t xcd = bid % kNumXcd, j = bid / kNumXcd;
  return xcd < rem ? xcd * (per + 1) + j : rem * (per + 1) + (xcd - rem) * per + j;
}

// Lanes of the wave whose 8-bit value equals this lane's, among `active`.  Every lane of
// `active` must execute the call (lanes outside the ballots would match a value of zero).
__device__ __forceinline__ uint64_t match_byte(uint32_t d, uint64_t active) {
  uint64_t m = active;
#pragma unroll
  for (int b = 0; b < 8; b++) {
    const uint64_t bal = __ballot((d >> b) & 1u);
    m &= ((d >> b) & 1u) ? bal : ~bal;
  }
  return m;
}

// List append with one atomic per wave: every lane of the wave must call it; lanes with
// `pred` get consecutive slots.  Returns the slot (undefined when !pred).
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool pred) {
  const uint64_t m = __ballot(pred);
  if (m == 0) return 0;
  const int leader = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if (__lane_id() == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
  base = (uint32_t)__shfl((int)base, leader, 64);
  return base + (uint32_t)__popcll(m & lanemask_lt());
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

}  // namespace bzg
