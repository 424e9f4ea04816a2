// origptr.hip -- A5 on the device.
//
// origPtr of block b = rank0[b] for an aperiodic block; 0 for a block of one repeated byte
// (no B* rotation, blocksort.c:1349); rank0[b] * k + r for a block w^k, where r is the copy
// index of rotation 0 (copyrank.cpp).  r has a closed form when the root w has exactly one
// B* offset (copyrank.cpp section 4), which covers every block cut from a long run of one
// byte (RLE1 makes it (c c c c n)^k); the device decides that case itself and writes origPtr
// without the host.  Blocks whose root has several B* offsets take r from the host model,
// which runs on the root bytes only (p bytes, copied once per block) in a host thread while
// the device sorts.
#include <map>
#include <mutex>
#include <string>

#include "common.h"
#include "copyrank.h"
#include "stages.h"

namespace bzg {
namespace {

constexpr int kT = 256;

// Number of B* offsets of the cyclic root blk[lo, lo + p): i is B* when w[i] < w[i+1] and the
// first symbol after the run that starts at i+1 is smaller than that run's symbol.
__global__ void __launch_bounds__(kT) k_root_bstar(const uint8_t* __restrict__ blk, const uint32_t* __restrict__ boff,
                                                   const uint32_t* __restrict__ period, uint32_t* __restrict__ bq) {
  __shared__ uint32_t cnt;
  const uint32_t b = blockIdx.x, lo = boff[b], n = boff[b + 1] - lo, p = period[b];
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  if (p >= 2 && p < n) {
    const uint8_t* w = blk + lo;
    uint32_t mine = 0;
    for (uint32_t i = threadIdx.x; i < p; i += kT) {
      const uint32_t j = i + 1 == p ? 0 : i + 1;
      const uint8_t c = w[j];
      if (w[i] >= c) continue;
      uint32_t t = j;  // a primitive root of length >= 2 holds two symbols: the scan ends
      do t = t + 1 == p ? 0 : t + 1;
      while (w[t] == c);
      mine += w[t] < c;
    }
    if (mine) atomicAdd(&cnt, mine);
  }
  __syncthreads();
  if (threadIdx.x == 0) bq[b] = cnt;
}

// copyrank.cpp section 4 (q == 1)
__device__ __forceinline__ uint32_t single_copy_rank(uint32_t p, uint32_t k) {
  const uint32_t s0 = k - 1 < 1024u ? k - 1 : 1024u;
  const uint32_t g = 1 + ((s0 > 8 && (p & 1)) ? s0 / 2 : 0);
  return (k > 8 && g == k / 2) ? 0 : g;
}

__global__ void __launch_bounds__(kT) k_origptr(const uint32_t* __restrict__ boff, const uint32_t* __restrict__ period,
                                                const uint32_t* __restrict__ bq, const uint32_t* __restrict__ rank0,
                                                const int32_t* __restrict__ host_r, uint32_t nb,
                                                uint32_t* __restrict__ origptr) {
  const uint32_t b = blockIdx.x * kT + threadIdx.x;
  if (b >= nb) return;
  const uint32_t n = boff[b + 1] - boff[b], p = period[b];
  uint32_t o;
  if (p >= n) {
    o = rank0[b];
  } else if (p == 1) {
    o = 0;
  } else {
    const uint32_t k = n / p;
    o = rank0[b] * k + (bq[b] == 1 ? single_copy_rank(p, k) : (uint32_t)host_r[b]);
  }
  origptr[b] = o;
}

// identical periodic roots (e.g. every block of a long constant input) resolve once; the memo
// holds at most kMemoBytes of root keys (a root can be ~450 KB) and bzg_release clears it
constexpr size_t kMemoBytes = 8u << 20;
std::mutex g_memo_mu;
std::map<std::pair<std::string, int32_t>, int32_t> g_memo;
size_t g_memo_bytes = 0;

int32_t memo_copy_rank(const uint8_t* w, int32_t p, int32_t k) {
  std::pair<std::string, int32_t> key(std::string((const char*)w, (size_t)p), k);
  {
    std::lock_guard<std::mutex> g(g_memo_mu);
    auto it = g_memo.find(key);
    if (it != g_memo.end()) return it->second;
  }
  const int32_t r = copy_rank(w, p, k);
  if ((size_t)p > kMemoBytes / 4) return r;  // too large to keep
  std::lock_guard<std::mutex> g(g_memo_mu);
  if (g_memo_bytes + (size_t)p > kMemoBytes || g_memo.size() >= 256) {
    g_memo.clear();
    g_memo_bytes = 0;
  }
  if (g_memo.emplace(std::move(key), r).second) g_memo_bytes += (size_t)p;
  return r;
}

}  // namespace

void copyrank_memo_clear() {
  std::lock_guard<std::mutex> g(g_memo_mu);
  g_memo.clear();
  g_memo_bytes = 0;
}

void copyrank_count_stage(Rle1Result& r, Workspace& ws, hipStream_t st) {
  const uint32_t B = r.nblocks;
  if (B == 0) return;
  r.bq = ws.u32("bq", B + 2);
  k_root_bstar<<<B, kT, 0, st>>>(r.blk, r.boff, r.period, r.bq);
  HIP_OK(hipGetLastError());
}

void copyrank_begin(const Rle1Result& r, const std::vector<uint32_t>& hboff, const std::vector<uint32_t>& hper,
                    const std::vector<uint32_t>& hbq, CopyRankJob& job, hipStream_t st) {
  const uint32_t nb = r.nblocks;
  std::vector<uint32_t> need;
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t n = hboff[b + 1] - hboff[b], p = hper[b];
    if (p >= 2 && p < n && hbq[b] != 1) need.push_back(b);
  }
  if (need.empty()) return;
  job.r.assign(nb, 0);
  size_t total = 0;
  for (uint32_t b : need) total += hper[b];
  job.roots.resize(total);
  size_t at = 0;
  for (uint32_t b : need) {  // the root only: p bytes per block
    HIP_OK(hipMemcpyAsync(job.roots.data() + at, r.blk + hboff[b], hper[b], hipMemcpyDeviceToHost, st));
    at += hper[b];
  }
  HIP_OK(hipStreamSynchronize(st));
  job.th = std::thread([&job, need, hboff, hper] {
    try {
      size_t pos = 0;
      for (uint32_t b : need) {
        const uint32_t n = hboff[b + 1] - hboff[b], p = hper[b];
        job.r[b] = memo_copy_rank(job.roots.data() + pos, (int32_t)p, (int32_t)(n / p));
        pos += p;
      }
    } catch (...) {
      job.err = std::current_exception();
    }
  });
}

void copyrank_finish(Workspace& ws, const Rle1Result& r, const uint32_t* rank0, uint32_t* origptr, CopyRankJob& job,
                     hipStream_t st) {
  const uint32_t nb = r.nblocks;
  if (nb == 0) return;
  int32_t* d_r = nullptr;
  if (job.th.joinable()) {
    job.th.join();
    if (job.err) {
      try {
        std::rethrow_exception(job.err);
      } catch (const CopyRankFailure&) {
        throw HipFailure(hipErrorInvalidValue);
      }
    }
    d_r = (int32_t*)ws.u32("copyrank_r", nb + 2);
    HIP_OK(hipMemcpyAsync(d_r, job.r.data(), 4ull * nb, hipMemcpyHostToDevice, st));  // job outlives the batch
  }
  k_origptr<<<ceil_div(nb, kT), kT, 0, st>>>(r.boff, r.period, r.bq, rank0, d_r, nb, origptr);
  HIP_OK(hipGetLastError());
}

CopyRankJob::~CopyRankJob() {
  if (th.joinable()) th.join();
}

}  // namespace bzg
