// origptr.hip -- A5 on the device.
//
// origPtr of block b = rank0[b] for an aperiodic block; 0 for a block of one repeated byte
// (no B* rotation, blocksort.c:1349); rank0[b] * k + r for a block w^k, where r is the copy
// index of rotation 0 (copyrank.cpp).  The device evaluates r itself in two closed forms:
//   * one B* offset per period (copyrank.cpp section 4): every block cut from a long run of one
//     byte (RLE1 makes it (c c c c n)^k), in k_origptr;
//   * several B* offsets in classes of pairwise different keys, the first class alone in its
//     (c0, c1) bucket, while the reference's rank-stage budget lasts (copyrank_cf.cpp), in
//     k_copyrank_cf, one workgroup per root.
// The roots left over take r from the host model (copyrank.cpp) on their p bytes.  That runs
// in a host function on a side stream (D2H of the roots and of the device's answers, the model
// for the roots the device left, H2D of the merged answers), so no host thread waits for the
// device: the origPtr kernel's stream waits for the side stream's event.
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

// copyrank_cf.cpp: classes of pairwise different keys, the first alone in its bucket.  One
// workgroup per listed root (q >= 2 B* offsets); out[b] = r, or -1 when the rule does not apply
// (the host model decides).
constexpr uint32_t kCT = 1024, kQMax = (uint32_t)kCopyRankQMax;
__device__ __forceinline__ int lg32d(uint32_t v) { return v == 0 ? -1 : 31 - (int)__builtin_clz(v); }
__global__ void __launch_bounds__(kCT) k_copyrank_cf(const uint8_t* __restrict__ blk, const uint32_t* __restrict__ boff,
                                                     const uint32_t* __restrict__ period, const uint32_t* __restrict__ bq,
                                                     const uint32_t* __restrict__ list, int32_t* __restrict__ out) {
  __shared__ uint32_t off[kQMax], bk[kQMax], gp[kQMax], rk[kQMax];
  __shared__ uint32_t sh[kCT / 64];
  __shared__ uint32_t fail, first;
  __shared__ unsigned long long work;
  const uint32_t b = list[blockIdx.x], lo = boff[b], n = boff[b + 1] - lo, p = period[b], q = bq[b];
  const uint32_t k = p ? n / p : 0;
  if (q < 2 || q > kQMax || p < 2 || k < 2 || (uint64_t)q * k > 0x7fffffffull || p > (uint32_t)kCopyRankPMax ||
      (int64_t)q * p > kCopyRankCmpMax) {  // (bounded comparisons: copyrank.h)
    if (threadIdx.x == 0) out[b] = -1;
    return;
  }
  const uint8_t* w = blk + lo;
  if (threadIdx.x == 0) {
    fail = 0;
    work = 0;
  }
  // B* offsets in increasing order (the rule of k_root_bstar)
  uint32_t base = 0;
  for (uint32_t i0 = 0; i0 < p; i0 += kCT) {
    const uint32_t i = i0 + threadIdx.x;
    bool is = false;
    if (i < p) {
      const uint32_t j = i + 1 == p ? 0 : i + 1;
      const uint8_t c = w[j];
      if (w[i] < c) {
        uint32_t t = j;
        do t = t + 1 == p ? 0 : t + 1;
        while (w[t] == c);
        is = w[t] < c;
      }
    }
    uint32_t tot;
    const uint32_t incl = block_incl_sum((uint32_t)is, sh, &tot);
    if (is && base + incl - 1 < kQMax) off[base + incl - 1] = i;
    base += tot;
  }
  __syncthreads();
  if (base != q) {  // (cannot happen: k_root_bstar counted the same offsets)
    if (threadIdx.x == 0) out[b] = -1;
    return;
  }
  for (uint32_t c = threadIdx.x; c < q; c += kCT) {
    bk[c] = ((uint32_t)w[off[c]] << 8) | w[off[c] + 1 == p ? 0 : off[c] + 1];
    gp[c] = (c + 1 < q ? off[c + 1] : off[0] + p) - off[c];
  }
  __syncthreads();
  // full key: bucket, then the substring characters 2 .. gap + 1 (a shorter equal prefix first)
  auto cmp = [&](uint32_t x, uint32_t y) -> int {
    if (bk[x] != bk[y]) return bk[x] < bk[y] ? -1 : 1;
    const uint32_t len = min(gp[x], gp[y]);
    uint32_t a = off[x] + 2, e = off[y] + 2;
    a = a >= p ? a - p : a;  // (off < p, p >= 2)
    e = e >= p ? e - p : e;
    a = a >= p ? a - p : a;
    e = e >= p ? e - p : e;
    for (uint32_t d = 0; d < len; d++) {
      const uint8_t ca = w[a], ce = w[e];
      if (ca != ce) return ca < ce ? -1 : 1;
      a = a + 1 == p ? 0 : a + 1;
      e = e + 1 == p ? 0 : e + 1;
    }
    return gp[x] == gp[y] ? 0 : gp[x] < gp[y] ? -1 : 1;
  };
  // processing order of the rank stage = key order; the keys must be pairwise different
  for (uint32_t c = threadIdx.x; c < q; c += kCT) {
    uint32_t less = 0;
    for (uint32_t d = 0; d < q; d++) {
      if (d == c) continue;
      const int o = cmp(d, c);
      less += o < 0;
      if (o == 0) fail = 1;
    }
    rk[c] = less;
    if (less == 0) first = c;
  }
  __syncthreads();
  // the first class alone in its bucket
  if (!fail)
    for (uint32_t c = threadIdx.x; c < q; c += kCT)
      if (c != first && bk[c] == bk[first]) fail = 1;
  __syncthreads();
  if (fail) {
    if (threadIdx.x == 0) out[b] = -1;
    return;
  }
  // work charged before the last group (copyrank_cf.cpp (c))
  const unsigned long long sortw = (unsigned long long)k * (unsigned long long)(lg32d(k) + 1);
  unsigned long long mine = 0;
  for (uint32_t c = threadIdx.x; c < q; c += kCT) {
    const uint32_t rc = rk[c];
    if (rc == 0 || rc == q - 1) continue;
    uint32_t h = 1, x = c + 1 == q ? 0 : c + 1;
    while (rk[x] > rc) {
      ++h;
      x = x + 1 == q ? 0 : x + 1;
    }
    mine += (unsigned long long)(h - 1) * k + sortw;
  }
  mine = wave_sum(mine);
  if (__lane_id() == 0 && mine) atomicAdd(&work, mine);
  __syncthreads();
  if (threadIdx.x != 0) return;
  const uint32_t m = q * k;
  const unsigned long long budget = (unsigned long long)(lg32d(m) * 2 / 3 + 1) * m;
  if (work + (unsigned long long)m >= budget) {
    out[b] = -1;
    return;
  }
  const uint32_t f = first;
  const uint32_t gap = gp[f];
  const bool wrapped = f == q - 1;
  const uint32_t s0 = min(wrapped ? k - 1 : k, 1024u);
  uint32_t g = (wrapped ? 1u : 0u) + ((s0 > 8 && (gap & 1)) ? s0 / 2 : 0u);
  if (k > 8 && (q & 1)) g = g == 0 ? k / 2 : g == k / 2 ? 0 : g;
  out[b] = (int32_t)g;
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

namespace {
// runs on the side stream's host-function thread: the host model for the roots the device
// left (pin_r < 0); no HIP calls here
void copyrank_host_fn(void* arg) {
  CopyRankJob& job = *static_cast<CopyRankJob*>(arg);
  size_t pos = 0;
  for (size_t i = 0; i < job.need.size(); i++) {
    const uint32_t b = job.need[i], p = job.per[i], n = job.len[i];
    if (job.pin_r[b] < 0) {
      try {
        job.pin_r[b] = memo_copy_rank(job.pin_roots + pos, (int32_t)p, (int32_t)(n / p));
        job.n_host++;
      } catch (...) {
        job.pin_r[b] = 0;
        job.failed = 1;
      }
    }
    pos += p;
  }
}
}  // namespace

void copyrank_begin(Workspace& ws, const Rle1Result& r, const std::vector<uint32_t>& hboff,
                    const std::vector<uint32_t>& hper, const std::vector<uint32_t>& hbq, CopyRankJob& job,
                    hipStream_t st) {
  const uint32_t nb = r.nblocks;
  job.need.clear();
  job.per.clear();
  job.len.clear();
  size_t total = 0;
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t n = hboff[b + 1] - hboff[b], p = hper[b];
    if (p >= 2 && p < n && hbq[b] != 1) {
      job.need.push_back(b);
      job.per.push_back(p);
      job.len.push_back(n);
      total += p;
    }
  }
  if (job.need.empty()) return;
  const uint32_t nn = (uint32_t)job.need.size();
  job.dev_r = reinterpret_cast<int32_t*>(ws.u32("copyrank_r", nb + 2));
  uint32_t* dlist = ws.u32("copyrank_list", nn + 2);
  HIP_OK(hipMemcpyAsync(dlist, job.need.data(), 4ull * nn, hipMemcpyHostToDevice, st));
  k_copyrank_cf<<<nn, kCT, 0, st>>>(r.blk, r.boff, r.period, r.bq, dlist, job.dev_r);
  HIP_OK(hipGetLastError());
  // side stream: the device's answers and the root bytes to pinned memory, the host model for
  // what is left, the merged answers back
  // (the part workspace's side stream orders this batch's use of its pinned buffers after the
  // previous batch's)
  job.side = ws.side_stream();
  job.pin_r = static_cast<int32_t*>(ws.pinned("copyrank_r", 4ull * (nb + 2)));
  job.pin_roots = static_cast<uint8_t*>(ws.pinned("copyrank_roots", total + 16));
  job.ev_cf = ws.side_event(0);
  job.ev_done = ws.side_event(1);
  HIP_OK(hipEventRecord(job.ev_cf, st));
  HIP_OK(hipStreamWaitEvent(job.side, job.ev_cf, 0));
  HIP_OK(hipMemcpyAsync(job.pin_r, job.dev_r, 4ull * nb, hipMemcpyDeviceToHost, job.side));
  size_t at = 0;
  for (size_t i = 0; i < job.need.size(); i++) {  // the root only: p bytes per block
    HIP_OK(hipMemcpyAsync(job.pin_roots + at, r.blk + hboff[job.need[i]], job.per[i], hipMemcpyDeviceToHost, job.side));
    at += job.per[i];
  }
  HIP_OK(hipLaunchHostFunc(job.side, copyrank_host_fn, &job));
  HIP_OK(hipMemcpyAsync(job.dev_r, job.pin_r, 4ull * nb, hipMemcpyHostToDevice, job.side));
  HIP_OK(hipEventRecord(job.ev_done, job.side));
}

void copyrank_finish(Workspace& ws, const Rle1Result& r, const uint32_t* rank0, uint32_t* origptr, CopyRankJob& job,
                     hipStream_t st) {
  (void)ws;
  const uint32_t nb = r.nblocks;
  if (nb == 0) return;
  if (job.ev_done) HIP_OK(hipStreamWaitEvent(st, job.ev_done, 0));  // a device-side wait
  k_origptr<<<ceil_div(nb, kT), kT, 0, st>>>(r.boff, r.period, r.bq, rank0, job.dev_r, nb, origptr);
  HIP_OK(hipGetLastError());
}

void copyrank_check(const CopyRankJob& job) {
  if (job.failed) throw HipFailure(hipErrorInvalidValue);
}

CopyRankJob::~CopyRankJob() {
  // the host function on the side stream reads this job (the stream, events and pinned
  // buffers belong to the part workspace)
  if (side) (void)hipStreamSynchronize(side);
}

}  // namespace bzg
