// engine.hip -- orchestration of the device pipeline and the bzg_* C ABI (include/bzg.h).
//
// Engines are pooled per device (EnginePool): every call leases one engine of the calling
// thread's current device, so host threads compress concurrently on separate HIP streams and
// device buffers.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <new>
#include <vector>
#include <cstring>
#include <exception>
#include <functional>
#include <future>
#include <mutex>
#include <thread>

#include "../../include/bzg.h"
#include "copyrank.h"
#include "stages.h"

#define BZ_OK 0
#define BZ_PARAM_ERROR (-2)
#define BZ_MEM_ERROR (-3)
#define BZ_OUTBUFF_FULL (-8)
#define BZ_CONFIG_ERROR (-9)

namespace bzg {

// ---------------------------------------------------------------- workspace
Workspace::~Workspace() {
  release_all();
  for (hipEvent_t& e : sev_)
    if (e) (void)hipEventDestroy(e);
  if (side_) (void)hipStreamDestroy(side_);
  if (handoff_) (void)hipEventDestroy(handoff_);
  if (mbox_) (void)hipHostFree(mbox_);
}

hipStream_t Workspace::side_stream() {
  if (!side_) HIP_OK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  return side_;
}

hipEvent_t Workspace::side_event(int k) {
  if (!sev_[k]) HIP_OK(hipEventCreateWithFlags(&sev_[k], hipEventDisableTiming));
  return sev_[k];
}

void* Workspace::pinned(const std::string& name, size_t bytes) {
  auto& b = pins_[name];
  if (b.second >= bytes) return b.first;
  if (b.first) {
    if (side_) HIP_OK(hipStreamSynchronize(side_));
    (void)hipHostFree(b.first);
    b.first = nullptr;
    b.second = 0;
  }
  const size_t grow = bytes + bytes / 4 + 64;
  HIP_OK(hipHostMalloc(&b.first, grow, hipHostMallocDefault));
  b.second = grow;
  return b.first;
}

// read_small: the words of up to four pieces to pinned host memory, then the flag (release at
// system scope after every word is visible)
constexpr uint32_t kMboxWords = 8192;
struct MboxPieces {
  const uint32_t* src[4];
  uint32_t nw[4], at[4], stride[4];
};
__global__ void __launch_bounds__(256) k_mbox(MboxPieces P, uint32_t* dst, uint32_t* flag, uint32_t seq) {
#pragma unroll
  for (int k = 0; k < 4; k++)
    for (uint32_t i = threadIdx.x; i < P.nw[k]; i += 256) dst[P.at[k] + i] = P.src[k][(size_t)i * P.stride[k]];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void Workspace::read_small(void* dst, const void* dev_src, size_t bytes, hipStream_t st) {
  read_small({SmallRead{dst, dev_src, bytes}}, st);
}

void Workspace::read_small(std::initializer_list<SmallRead> reads, hipStream_t st) {
  MboxPieces P{};
  uint32_t total = 0;
  bool fast = reads.size() <= 4;
  int k = 0;
  for (const SmallRead& r : reads) {
    const size_t nw = (r.bytes + 3) / 4;
    fast = fast && (reinterpret_cast<uintptr_t>(r.src) & 3u) == 0 && total + nw <= kMboxWords;
    if (k < 4) {
      P.src[k] = static_cast<const uint32_t*>(r.src);
      P.nw[k] = (uint32_t)nw;
      P.at[k] = total;
      P.stride[k] = std::max(r.stride, 1u);
    }
    total += (uint32_t)std::min<size_t>(nw, kMboxWords + 1);
    k++;
  }
  // (a strided piece's words one copy each)
  auto copy_async = [&](const SmallRead& r) {
    if (r.stride <= 1) {
      HIP_OK(hipMemcpyAsync(r.dst, r.src, r.bytes, hipMemcpyDeviceToHost, st));
      return;
    }
    for (size_t i = 0; i < r.bytes / 4; i++)
      HIP_OK(hipMemcpyAsync(static_cast<uint32_t*>(r.dst) + i, static_cast<const uint32_t*>(r.src) + i * r.stride, 4,
                            hipMemcpyDeviceToHost, st));
  };
  if (!fast) {
    for (const SmallRead& r : reads) copy_async(r);
    HIP_OK(hipStreamSynchronize(st));
    return;
  }
  if (!mbox_) {
    HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&mbox_), (kMboxWords + 16) * 4, hipHostMallocCoherent));
    HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&mbox_dev_), mbox_, 0));
    mbox_[kMboxWords] = 0;
  }
  const uint32_t seq = ++mseq_ == 0 ? ++mseq_ : mseq_;
  k_mbox<<<1, 256, 0, st>>>(P, mbox_dev_, mbox_dev_ + kMboxWords, seq);
  HIP_OK(hipGetLastError());
  uint32_t* flag = mbox_ + kMboxWords;
  // spin while the answer is expected within microseconds (the sort's list sizes); a wait
  // longer than the spin budget (a whole batch still queued) blocks in the runtime instead of
  // keeping a core busy beside the other host threads
  constexpr uint64_t kSpinBudget = 1u << 15;  // about 1 ms
  for (uint64_t spins = 1;; spins++) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) break;
    if (spins == kSpinBudget) {
      HIP_OK(hipStreamSynchronize(st));  // k_mbox is the stream's last operation
      if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) break;
    }
    if ((spins & 1023) == 0) {  // a fault or an error on the stream ends the wait
      const hipError_t e = hipStreamQuery(st);
      if (e == hipSuccess) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) break;
        for (const SmallRead& r : reads) copy_async(r);  // (not expected)
        HIP_OK(hipStreamSynchronize(st));
        return;
      }
      if (e != hipErrorNotReady) HIP_OK(e);
    }
    __builtin_ia32_pause();
  }
  k = 0;
  for (const SmallRead& r : reads) std::memcpy(r.dst, mbox_ + P.at[k++], r.bytes);
}

void Workspace::set_stream(hipStream_t s) {
  if (s == stream_) return;
  // no throw: Lease's destructor hands the workspaces back to the engine's own stream.  The new
  // stream must not run ahead of work still queued on the old one (a later free or growth on
  // the new stream would release a buffer in use): an event when possible, else a host wait.
  if (!bufs_.empty()) {
    bool ordered = false;
    if (handoff_ || hipEventCreateWithFlags(&handoff_, hipEventDisableTiming) == hipSuccess)
      ordered = hipEventRecord(handoff_, stream_) == hipSuccess && hipStreamWaitEvent(s, handoff_, 0) == hipSuccess;
    if (!ordered) (void)hipStreamSynchronize(stream_);
  }
  stream_ = s;
}

void Workspace::drop(Buf& b) {
  if (!b.p) return;
  if (b.async)
    (void)hipFreeAsync(b.p, stream_);
  else
    (void)hipFree(b.p);
  total_ -= b.bytes;
  b.p = nullptr;
  b.bytes = 0;
}

void Workspace::release_all() {
  if (!pins_.empty()) {
    if (side_) (void)hipStreamSynchronize(side_);
    for (auto& kv : pins_)
      if (kv.second.first) (void)hipHostFree(kv.second.first);
    pins_.clear();
  }
  bool any_async = false;
  for (auto& kv : bufs_) {
    any_async |= kv.second.async && kv.second.p;
    drop(kv.second);
  }
  bufs_.clear();
  total_ = 0;
  if (any_async) (void)hipStreamSynchronize(stream_);
  if (crc_) (void)hipFree(crc_);
  if (xp2_) (void)hipFree(xp2_);
  crc_ = xp2_ = nullptr;
}

void* Workspace::get(const std::string& name, size_t bytes, bool zero) {
  bytes = std::max<size_t>(bytes, 64);
  Buf& b = bufs_[name];
  if (b.bytes >= bytes) return b.p;
  static const bool sync_free = getenv("BZG_WS_SYNC_FREE") != nullptr;
  const bool async = stream_ != nullptr && !sync_free;
  if (b.p) {
    // the old buffer may still be read by work queued on this workspace's stream: an async
    // free is ordered after it; a synchronous one waits for that stream only
    if (!b.async && stream_) HIP_OK(hipStreamSynchronize(stream_));
    else if (!b.async) HIP_OK(hipDeviceSynchronize());
    drop(b);
  }
  const size_t grow = bytes + bytes / 8;  // headroom so small growth does not realloc
  void* p = nullptr;
  const hipError_t e = async ? hipMallocAsync(&p, grow, stream_) : hipMalloc(&p, grow);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky error of the failed allocation
    throw HipFailure(hipErrorOutOfMemory);
  }
  b.p = p;
  b.bytes = grow;
  b.async = async;
  total_ += grow;
  if (zero) HIP_OK(stream_ ? hipMemsetAsync(p, 0, grow, stream_) : hipMemset(p, 0, grow));
  return b.p;
}

static uint32_t host_gf_mul(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int i = 31; i >= 0; i--) {
    r = (r & 0x80000000u) ? (r << 1) ^ 0x04C11DB7u : (r << 1);
    if ((b >> i) & 1u) r ^= a;
  }
  return r;
}

const uint32_t* Workspace::crc_table() {
  if (!crc_) {
    uint32_t t[256];
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t r = i << 24;
      for (int k = 0; k < 8; k++) r = (r & 0x80000000u) ? (r << 1) ^ 0x04C11DB7u : (r << 1);
      t[i] = r;
    }
    HIP_OK(hipMalloc(&crc_, sizeof(t)));
    HIP_OK(hipMemcpy(crc_, t, sizeof(t), hipMemcpyHostToDevice));
  }
  return crc_;
}

const uint32_t* Workspace::xpow2_table() {
  if (!xp2_) {
    uint32_t t[48];
    t[0] = 0x100u;  // x^8
    for (int k = 1; k < 48; k++) t[k] = host_gf_mul(t[k - 1], t[k - 1]);
    HIP_OK(hipMalloc(&xp2_, sizeof(t)));
    HIP_OK(hipMemcpy(xp2_, t, sizeof(t), hipMemcpyHostToDevice));
  }
  return xp2_;
}

// ---------------------------------------------------------------- engine
// An engine is one device's HIP streams, events and workspaces.  It serves one call at a
// time.  Engines live in a pool keyed by device (EnginePool below): a call leases a free
// engine of its device, creates one while the device has fewer than the cap, or waits.
// Streams of several host threads therefore run on separate HIP streams and device buffers,
// as the reference keeps all compression state per bz_stream (bzlib.c:144-207).
struct Engine {
  static constexpr int kSortStreams = 3;
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t sstream[kSortStreams] = {};  // block sorts of the batch's parts
  hipStream_t cstream = nullptr;             // host <-> device copies of the pipelined host calls
  Workspace ws;
  std::vector<std::unique_ptr<Workspace>> pws;  // one per part of a batch
  std::vector<hipEvent_t> psorted;              // per part: its sort is done
  hipEvent_t ev_rle;  // the sort streams start after RLE1

  explicit Engine(int dev) : device(dev) {
    HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    for (auto& x : sstream) HIP_OK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&ev_rle, hipEventDisableTiming));
    ws.set_stream(stream);
  }

  // Back to the engine's own stream once a call is over: a caller's stream may be destroyed
  // after the call, and later growth or release must not be ordered on it.
  void own_streams() {
    ws.set_stream(stream);
    ws2.set_stream(stream);
    for (auto& w : pws) w->set_stream(stream);
  }
  void release_idle() {
    own_streams();
    ws.release_all();
    ws2.release_all();
    for (auto& w : pws) w->release_all();
  }

  // One part of a batch: consecutive blocks [b0, b1) with their own device view (block
  // offsets relative to the part), workspace and results.
  struct Part {
    uint32_t b0 = 0, b1 = 0;
    Rle1Result r;
    std::vector<uint32_t> hboff, hper, hbq, hqp;
    Workspace* w = nullptr;
    CopyRankJob a5;
    SortStats ss;
    MtfResult m;
    CodeTables t;
    float sort_ms = 0;
  };

  Workspace* part_ws(size_t p) {
    while (pws.size() <= p) pws.emplace_back(new Workspace());
    while (psorted.size() <= p) {
      hipEvent_t e;
      HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      psorted.push_back(e);
    }
    return pws[p].get();
  }

  // Parts per batch and concurrent sort streams (BZG_PARTS / BZG_SORT_STREAMS).  Batches of
  // fewer than 64 blocks are one part on one stream.
  static bool split_tables() {  // BZG_SPLIT_TABLES=0: one stream for the table optimisation
    static const bool v = cfg("BZG_SPLIT_TABLES", 1, 0, 1) != 0;
    return v;
  }
  static int cfg(const char* name, int dflt, int lo, int hi) {
    const char* e = getenv(name);
    return std::min(hi, std::max(lo, e ? atoi(e) : dflt));
  }

  // ---- one batch, in two stages -------------------------------------------------------
  // front: RLE1 and the block sorts (origPtr included); back: MTF, the table optimisation and
  // the packing.  batch() runs both on the caller's stream.  A multi-batch input pipelines them
  // (compress below): the back stage of batch j (its own workspace slot and streams) runs
  // beside the front stage of batch j + 1, which needs only batch j's consumed input.
  //
  // The blocks are cut into parts.  Each part is sorted on one of the sort streams by its own
  // host thread (the sorter synchronises with the host between passes, so several parts keep
  // the device busy); origPtr of a part's blocks follows its sort on the same stream.
  struct SlotEvents {  // timing and side-stream events of one workspace slot
    hipEvent_t ev[6] = {};
    hipEvent_t tev[3] = {};
    hipEvent_t crc_in = nullptr, crc_out = nullptr;
    hipEvent_t sorted = nullptr;  // the front stage is complete on every stream it used
    void create() {
      if (crc_in) return;
      for (auto& e : ev) HIP_OK(hipEventCreate(&e));
      for (auto& e : tev) HIP_OK(hipEventCreate(&e));
      HIP_OK(hipEventCreateWithFlags(&crc_in, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&crc_out, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&sorted, hipEventDisableTiming));
    }
  };
  struct BatchCtx {
    Workspace* w = nullptr;
    SlotEvents* e = nullptr;
    int level = 9;
    bool end_seg = false, tail_merge = false, trailer = false;
    Rle1Result r;
    uint32_t nb = 0, nparts = 0;
    std::vector<uint32_t> hboff, hper, hbq, hqp;
    std::unique_ptr<Part[]> parts;
    uint32_t* origptr = nullptr;
    uint8_t* bwt = nullptr;
    uint64_t sort_iters = 0, sort_unsorted = 0;
    uint64_t consumed = 0;
  };

  void front(BatchCtx& c, const uint8_t* d_in, uint64_t n, unsigned flags, int level, hipStream_t s) {
    Workspace& W = *c.w;
    SlotEvents& E = *c.e;
    c.level = level;
    c.end_seg = flags & BZG_FLAG_END_SEGMENT;
    c.tail_merge = (flags & BZG_FLAG_TAIL_MERGE) && c.end_seg;
    c.trailer = (flags & BZG_FLAG_TRAILER) && c.end_seg;
    W.set_stream(s);
    HIP_OK(hipEventRecord(E.ev[0], s));
    Rle1Result& r = c.r;
    // the block CRCs run on the last sort stream (idle at the default two sort streams; with
    // three it only queues behind that stream's sorts) and overlap the sort
    hipStream_t crc_st = sstream[kSortStreams - 1];  // (profiles/r05_ab_crc_side.txt)
    // on an error path the CRC / in-use kernels may still be in flight on crc_st when the next
    // call frees or regrows the workspace on s: wait for them before the exception leaves
    struct SideJoin {
      hipStream_t side;
      ~SideJoin() {
        if (std::uncaught_exceptions() > 0) (void)hipStreamSynchronize(side);
      }
    } side_join{crc_st};
    rle1_stage(W, d_in, n, level, c.end_seg, c.tail_merge, r, s, crc_st, E.crc_in, E.crc_out);
    HIP_OK(hipEventRecord(E.ev[1], s));
    c.consumed = c.end_seg ? n : r.consumed;
    const uint32_t nb = c.nb = r.nblocks;
    c.origptr = W.u32("origptr", nb + 2);
    c.hboff.assign(nb + 1, 0u);
    c.hper.assign(nb, 0u);
    c.hbq.assign(nb, 0u);
    c.hqp.assign(nb, 0u);
    if (nb == 0) {
      HIP_OK(hipEventRecord(E.sorted, s));
      return;
    }
    W.read_small({{c.hboff.data(), r.boff, 4ull * (nb + 1)}, {c.hper.data(), r.period, 4ull * nb},
                  {c.hbq.data(), r.bq, 4ull * nb}, {c.hqp.data(), r.qper, 4ull * nb}},
                 s);
    uint8_t* bwt = c.bwt = W.u8("bwt", c.hboff[nb] + 16);
    uint32_t* rank0 = W.u32("rank0", nb + 2);
    uint32_t* origptr = c.origptr;
    static const bool one_stream = getenv("BZG_ONE_STREAM") != nullptr;  // per-kernel profiling
    const int want = nb < 64 || one_stream ? 1 : cfg("BZG_PARTS", 2, 1, 16);
    const uint32_t K = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)want, nb / 16));
    const int S = nb < 64 || one_stream ? 1 : std::min<int>((int)K, cfg("BZG_SORT_STREAMS", 2, 1, kSortStreams));
    c.parts.reset(new Part[K]);
    c.nparts = K;
    Part* parts = c.parts.get();
    for (uint32_t p = 0; p < K; p++) {
      Part& P = parts[p];
      P.b0 = (uint32_t)((uint64_t)nb * p / K);
      P.b1 = (uint32_t)((uint64_t)nb * (p + 1) / K);
      const uint32_t pn = P.b1 - P.b0, base = c.hboff[P.b0];
      P.w = part_ws(p);
      P.w->set_stream(s);
      P.hboff.assign(c.hboff.begin() + P.b0, c.hboff.begin() + P.b1 + 1);
      for (auto& x : P.hboff) x -= base;
      P.hper.assign(c.hper.begin() + P.b0, c.hper.begin() + P.b1);
      P.hbq.assign(c.hbq.begin() + P.b0, c.hbq.begin() + P.b1);
      P.hqp.assign(c.hqp.begin() + P.b0, c.hqp.begin() + P.b1);
      P.r = r;
      P.r.nblocks = pn;
      P.r.blk = r.blk + base;
      P.r.boff = P.w->u32("part_boff", pn + 2);
      HIP_OK(hipMemcpyAsync(P.r.boff, P.hboff.data(), 4ull * (pn + 1), hipMemcpyHostToDevice, s));
      P.r.binst = nullptr;
      P.r.bcrc = r.bcrc + P.b0;
      P.r.inuse = r.inuse + 8ull * P.b0;
      P.r.ninuse = r.ninuse + P.b0;
      P.r.period = r.period + P.b0;
      P.r.bq = r.bq + P.b0;
      P.r.qper = r.qper + P.b0;
    }
    HIP_OK(hipEventRecord(ev_rle, s));  // the sort streams start after RLE1 and the views
    std::vector<std::promise<void>> sorted(K);
    std::vector<std::future<void>> sorted_f;
    for (auto& x : sorted) sorted_f.push_back(x.get_future());
    // raised right after a part's promise is settled: the main thread spins on it rather
    // than sleeping in the future (a wake-up took ~50 us of idle device per part)
    std::unique_ptr<std::atomic<int>[]> settled(new std::atomic<int>[K]);
    for (uint32_t p = 0; p < K; p++) settled[p].store(0);
    const int dev = device;
    auto sorter = [&, dev](int t) {
      try {
        HIP_OK(hipSetDevice(dev));  // the current device is per host thread
      } catch (...) {
        for (uint32_t p = (uint32_t)t; p < K; p += (uint32_t)S) {
          sorted[p].set_exception(std::current_exception());
          settled[p].store(1, std::memory_order_release);
        }
        return;
      }
      hipStream_t ss = S == 1 ? s : sstream[t];
      bool failed = false;
      for (uint32_t p = (uint32_t)t; p < K; p += (uint32_t)S) {
        if (failed) {
          sorted[p].set_exception(std::make_exception_ptr(HipFailure(hipErrorUnknown)));
          settled[p].store(1, std::memory_order_release);
          continue;
        }
        try {
          Part& P = parts[p];
          P.w->set_stream(ss);
          if (ss != s) HIP_OK(hipStreamWaitEvent(ss, ev_rle, 0));
          copyrank_begin(*P.w, P.r, P.hboff, P.hper, P.hbq, P.a5, ss);  // (side stream: overlaps the sort)
          bwt_stage(*P.w, P.r, P.hboff, P.hper, bwt + c.hboff[P.b0], rank0 + P.b0, &P.ss, ss, P.hqp.data());
          copyrank_finish(*P.w, P.r, rank0 + P.b0, origptr + P.b0, P.a5, ss);
          HIP_OK(hipEventRecord(psorted[p], ss));
          sorted[p].set_value();
        } catch (...) {
          failed = true;
          sorted[p].set_exception(std::current_exception());
        }
        settled[p].store(1, std::memory_order_release);
      }
    };
    std::vector<std::thread> th;
    std::exception_ptr err;
    try {
      // this thread sorts the first stream's parts itself (one thread fewer to start, and it
      // does not sit idle)
      for (int t = 1; t < S; t++) th.emplace_back(sorter, t);
      sorter(0);
      for (uint32_t p = 0; p < K; p++) {
        if (S > 1)
          while (!settled[p].load(std::memory_order_acquire)) __builtin_ia32_pause();
        sorted_f[p].get();
        HIP_OK(hipStreamWaitEvent(s, psorted[p], 0));
      }
      HIP_OK(hipStreamWaitEvent(s, E.crc_out, 0));  // in-use maps and block CRCs (side stream)
      HIP_OK(hipEventRecord(E.sorted, s));
    } catch (...) {
      err = std::current_exception();
    }
    for (auto& x : th) x.join();
    if (err) std::rethrow_exception(err);
    for (uint32_t p = 0; p < K; p++) {
      c.sort_iters = std::max<uint64_t>(c.sort_iters, (uint64_t)parts[p].ss.iterations);
      c.sort_unsorted += parts[p].ss.unsorted_elems;
    }
  }

  // MTF, tables and packing of a front-staged batch on stream s (s2: the second table stream,
  // or null).  `before_emit` (optional) runs on this thread right before the packing, which
  // needs the stream state the previous batch leaves.
  void back(BatchCtx& c, bzg_stream_state* st, uint8_t* d_out, uint64_t out_cap, uint64_t* out_bytes, hipStream_t s,
            hipStream_t s2, bzg_stats& last, const std::function<void()>& before_emit = nullptr) {
    Workspace& W = *c.w;
    SlotEvents& E = *c.e;
    W.set_stream(s);
    HIP_OK(hipStreamWaitEvent(s, E.sorted, 0));
    const uint32_t nb = c.nb;
    Part* parts = c.parts.get();
    Part one;  // the whole batch from here on
    float mtf_ms = 0, tab_ms = 0;
    if (nb > 0) {
      HIP_OK(hipEventRecord(E.tev[0], s));
      one.b0 = 0;
      one.b1 = nb;
      one.r = c.r;
      one.hboff = c.hboff;
      one.w = &W;
      mtf_stage(W, c.r, c.bwt, nb, c.hboff[nb], one.m, s, &c.hboff);
      HIP_OK(hipEventRecord(E.tev[1], s));
      code_tables(W, c.r, one.m, nb, one.t, s, s2);
      HIP_OK(hipEventRecord(E.tev[2], s));  // (timings and the A5 check once the batch is done, below)
    }
    HIP_OK(hipEventRecord(E.ev[2], s));
    if (before_emit) before_emit();
    StreamCarry cy;
    cy.combined_crc = st->combined_crc;
    cy.carry_bits = st->carry_bits;
    cy.carry_byte = st->carry_byte;
    cy.header_done = st->header_done;
    std::vector<CodePart> cp;
    if (nb > 0) cp.push_back(CodePart{&one.r, &one.m, &one.t, c.origptr, nb});
    *out_bytes = code_emit(W, cp, c.level, c.trailer, cy, d_out, out_cap, s);
    HIP_OK(hipEventRecord(E.ev[4], s));
    // the batch's end: the MTF symbol counts (a statistic) come back through the spinning
    // small read, which is also the wait for the batch (a sleeping event wait cost ~40 us)
    std::vector<uint32_t> nm(nb);
    if (nb > 0)
      W.read_small(nm.data(), one.m.nmtf, 4ull * nb, s);
    else
      HIP_OK(hipEventSynchronize(E.ev[4]));
    if (nb > 0) {
      for (uint32_t p = 0; p < c.nparts; p++) copyrank_check(parts[p].a5);
      (void)hipEventElapsedTime(&mtf_ms, E.tev[0], E.tev[1]);
      (void)hipEventElapsedTime(&tab_ms, E.tev[1], E.tev[2]);
    }
    st->combined_crc = cy.combined_crc;
    st->carry_bits = cy.carry_bits;
    st->carry_byte = cy.carry_byte;
    st->header_done = cy.header_done ? 1 : 0;
    st->blocks_done += nb;
    last = bzg_stats{};
    float pipe_ms = 0, emit_ms = 0;
    (void)hipEventElapsedTime(&last.rle1_ms, E.ev[0], E.ev[1]);
    (void)hipEventElapsedTime(&pipe_ms, E.ev[1], E.ev[2]);
    (void)hipEventElapsedTime(&emit_ms, E.ev[2], E.ev[4]);
    (void)hipEventElapsedTime(&last.total_ms, E.ev[0], E.ev[4]);
    // the BWT figure is the sort pipeline up to the tables' end minus MTF and the tables
    last.mtf_ms = mtf_ms;
    last.code_ms = tab_ms + emit_ms;
    last.bwt_ms = std::max(0.f, pipe_ms - mtf_ms - tab_ms);
    last.nblocks = nb;
    last.sort_iterations = (int)c.sort_iters;
    last.rle_bytes = nb ? c.hboff[nb] : 0;
    last.sort_unsorted = c.sort_unsorted;
    for (uint32_t p = 0; p < c.nparts; p++) {
      last.a5_roots += (uint32_t)parts[p].a5.need.size();
      last.a5_host += parts[p].a5.n_host;
    }
    for (uint32_t x : nm) last.mtf_symbols += x;
  }

  // Compress one batch on stream s.  Throws HipFailure on device errors, OutBuffFull when
  // out_cap is short.
  SlotEvents slot_ev[2];
  Workspace ws2;  // the second workspace slot of pipelined batches
  void batch(const uint8_t* d_in, uint64_t n, unsigned flags, bzg_stream_state* st, uint8_t* d_out,
             uint64_t out_cap, uint64_t* out_bytes, uint64_t* consumed, hipStream_t s, bzg_stats& last) {
    slot_ev[0].create();
    BatchCtx c;
    c.w = &ws;
    c.e = &slot_ev[0];
    front(c, d_in, n, flags, st->level, s);
    back(c, st, d_out, out_cap, out_bytes, s, split_tables() ? sstream[0] : nullptr, last);
    *consumed = c.consumed;
  }

  // bzg_compress_device's contract: inputs larger than max_batch() are cut into batches; the
  // non-final batches emit complete blocks and the rest is resubmitted.
  void compress(const uint8_t* d_in, uint64_t n, unsigned flags, bzg_stream_state* st, uint8_t* d_out,
                uint64_t out_cap, uint64_t* out_bytes, uint64_t* consumed, hipStream_t s, bzg_stats& last);
  // Host-call hooks of the pipelined batches: `ends` (ascending input offsets, the last = n)
  // cuts the batches at the pieces of a staged upload; wait_input(end) makes the caller's
  // stream wait for the upload of [0, end); on_output(off, len) runs once a batch's coded
  // bytes [off, off + len) of the output are final (on the back-stage thread, in batch order).
  struct PipeHooks {
    std::vector<uint64_t> ends;
    std::function<void(uint64_t)> wait_input;
    std::function<void(uint64_t, uint64_t)> on_output;
  };
  void compress_pipelined(const uint8_t* d_in, uint64_t n, unsigned flags, bzg_stream_state* st, uint8_t* d_out,
                          uint64_t out_cap, uint64_t* out_bytes, uint64_t* consumed, hipStream_t s, bzg_stats& last,
                          const PipeHooks* hooks = nullptr);
};

// Largest batch handled in one pass: keeps every block/slot offset in 32 bits.  BZG_MAX_BATCH
// lowers it (tests: several pipelined batches from a small input).
static constexpr uint64_t kMaxBatchLimit = 1500ull * 1000 * 1000;
static uint64_t max_batch() {
  static const uint64_t v = std::min<uint64_t>(kMaxBatchLimit, (uint64_t)std::max(1000000ll, env_ll("BZG_MAX_BATCH", (long long)kMaxBatchLimit)));
  return v;
}

static void add_stats(bzg_stats& acc, const bzg_stats& one) {
  acc.rle1_ms += one.rle1_ms;
  acc.bwt_ms += one.bwt_ms;
  acc.mtf_ms += one.mtf_ms;
  acc.code_ms += one.code_ms;
  acc.total_ms += one.total_ms;
  acc.nblocks += one.nblocks;
  acc.sort_iterations = std::max(acc.sort_iterations, one.sort_iterations);
  acc.rle_bytes += one.rle_bytes;
  acc.sort_unsorted += one.sort_unsorted;
  acc.mtf_symbols += one.mtf_symbols;
  acc.a5_roots += one.a5_roots;
  acc.a5_host += one.a5_host;
}

void Engine::compress(const uint8_t* d_in, uint64_t n, unsigned flags, bzg_stream_state* st, uint8_t* d_out,
                      uint64_t out_cap, uint64_t* out_bytes, uint64_t* consumed, hipStream_t s, bzg_stats& last) {
  const bool pipe = cfg("BZG_BATCH_PIPE", 1, 0, 1) != 0;  // BZG_BATCH_PIPE=0: batches one after another (per call)
  const uint64_t batch_max = max_batch();
  if (pipe && n > batch_max) return compress_pipelined(d_in, n, flags, st, d_out, out_cap, out_bytes, consumed, s, last);
  ws.set_stream(s);
  uint64_t done_in = 0, done_out = 0;
  bzg_stats acc{};
  for (;;) {
    const uint64_t left = n - done_in;
    const bool last_piece = left <= batch_max;
    const uint64_t take = last_piece ? left : batch_max;
    const unsigned f = last_piece ? flags : 0u;
    uint64_t ob = 0, cons = 0;
    bzg_stats one{};
    // the packer ORs 32-bit words: a batch whose destination is not 4-byte aligned (any batch
    // after the first of a split input, or a caller's odd pointer) is coded into an aligned
    // workspace buffer and copied behind the previous batch's bytes
    uint8_t* dst = d_out + done_out;
    uint64_t cap = out_cap - done_out;
    const bool misaligned = ((uintptr_t)dst & 3u) != 0;
    uint8_t* bdst = dst;
    if (misaligned) {
      cap = std::min<uint64_t>(cap, bzg_bound(take));
      bdst = ws.u8("batch_out", cap + 16);
    }
    batch(d_in + done_in, take, f, st, bdst, cap, &ob, &cons, s, one);
    if (misaligned && ob) {
      HIP_OK(hipMemcpyAsync(dst, bdst, ob, hipMemcpyDeviceToDevice, s));
      HIP_OK(hipStreamSynchronize(s));
    }
    add_stats(acc, one);
    done_in += cons;
    done_out += ob;
    if (last_piece) break;
    if (cons == 0) throw HipFailure(hipErrorUnknown);  // cannot happen: a batch holds many blocks
  }
  *out_bytes = done_out;
  *consumed = done_in;
  last = acc;
}

// Batches of a multi-batch input, pipelined over two workspace slots: the front stage (RLE1,
// sorts) of batch j + 1 runs on the caller's stream and the sort streams while the back stage
// (MTF, tables, packing) of batch j runs on its slot's own streams from a second host thread.
// The back stages pack in batch order (each needs the stream state and the output position the
// previous one leaves); the front stage of batch j + 2 reuses slot j % 2 once batch j is done.
// MTF is VALU-bound and the sorts wait on gathers, so the two overlap well (4 GiB of PRNG bytes,
// three batches: profiles/r06_*).  The bytes equal the sequential batches' (the same stages on
// the same inputs).
void Engine::compress_pipelined(const uint8_t* d_in, uint64_t n, unsigned flags, bzg_stream_state* st,
                                uint8_t* d_out, uint64_t out_cap, uint64_t* out_bytes, uint64_t* consumed,
                                hipStream_t s, bzg_stats& last, const PipeHooks* hooks) {
  for (int k = 0; k < 2; k++) slot_ev[k].create();
  // The back stages run on the CRC side stream, one stream, no table split.  A process has 4
  // hardware queues (GPU_MAX_HW_QUEUES) and streams share them round-robin in creation order:
  // the caller's and the engine's own stream, the two sort streams and the CRC stream take all
  // four, and a back stage on a fifth stream shared a sort stream's queue, so it ran behind the
  // next batch's sorts instead of beside them (config 5: no gain at all).  On the CRC stream it
  // only delays the next batch's block CRCs, which nothing before that batch's back stage reads.
  hipStream_t bs = sstream[kSortStreams - 1];
  const uint64_t batch_max = max_batch();
  Workspace* slot_ws[2] = {&ws, &ws2};
  ws.set_stream(s);
  ws2.set_stream(s);
  std::unique_ptr<BatchCtx> ctx[2];
  std::thread backer;  // the back stage of the previous batch
  std::exception_ptr back_err;
  uint64_t done_in = 0, done_out = 0;
  size_t piece = 0;  // hooks->ends[piece]: the end of the next input piece
  bzg_stats acc{};
  std::mutex mu;
  auto join_back = [&] {
    if (backer.joinable()) backer.join();
    if (back_err) std::rethrow_exception(back_err);
  };
  try {
    for (uint32_t j = 0;; j++) {
      // a batch ends at the next piece end (the previous batch's leftover, less than a block,
      // joins it) or after batch_max bytes
      uint64_t end = std::min(n, done_in + batch_max);
      if (hooks && piece < hooks->ends.size() && hooks->ends[piece] <= end) end = hooks->ends[piece++];
      const bool last_piece = end == n;
      const uint64_t take = end - done_in;
      if (hooks && hooks->wait_input) hooks->wait_input(end);
      const int k = (int)(j & 1);
      // slot k was batch j - 2's: its back stage ended before batch j - 1's began (below)
      ctx[k].reset(new BatchCtx);
      BatchCtx& c = *ctx[k];
      c.w = slot_ws[k];
      c.e = &slot_ev[k];
      front(c, d_in + done_in, take, last_piece ? flags : 0u, st->level, s);
      if (!last_piece && c.consumed == 0) throw HipFailure(hipErrorUnknown);  // a batch holds many blocks
      // the previous batch's back stage must have packed before this one packs: this thread
      // waits for it here, then hands this batch's back stage to a new thread
      join_back();
      uint8_t* dst = d_out + done_out;
      const uint64_t dcap = out_cap - done_out;
      // the slot moves to the back stage's stream here, before the next front stage queues
      // anything on s (a handoff made later from the back thread would order the back stage
      // behind that work too)
      c.w->set_stream(bs);
      HIP_OK(hipStreamWaitEvent(bs, c.e->sorted, 0));
      const uint64_t take_in = c.consumed;
      done_in += take_in;
      backer = std::thread([&, k, dst, dcap, take] {
        try {
          HIP_OK(hipSetDevice(device));
          BatchCtx& b = *ctx[k];
          const bool misaligned = ((uintptr_t)dst & 3u) != 0;
          uint64_t cap = dcap;
          uint8_t* bdst = dst;
          if (misaligned) {
            b.w->set_stream(bs);
            cap = std::min<uint64_t>(cap, bzg_bound(take));
            bdst = b.w->u8("batch_out", cap + 16);
          }
          uint64_t ob = 0;
          bzg_stats one{};
          back(b, st, bdst, cap, &ob, bs, nullptr, one);
          if (misaligned && ob) {
            HIP_OK(hipMemcpyAsync(dst, bdst, ob, hipMemcpyDeviceToDevice, bs));
            HIP_OK(hipStreamSynchronize(bs));
          }
          uint64_t off;
          {
            std::lock_guard<std::mutex> g(mu);
            add_stats(acc, one);
            off = done_out;
            done_out += ob;
          }
          if (hooks && hooks->on_output) hooks->on_output(off, ob);
        } catch (...) {
          back_err = std::current_exception();
        }
      });
      if (last_piece) break;
    }
    join_back();
  } catch (...) {
    if (backer.joinable()) backer.join();
    (void)hipStreamSynchronize(bs);
    throw;
  }
  // the slots' workspaces go back to the caller's stream order: later growth or release by the
  // next call is ordered after the back streams' work (already complete: the back stages
  // ended with a host wait)
  ws2.set_stream(stream);
  *out_bytes = done_out;
  *consumed = done_in;
  last = acc;
}

// Makes `dev` the calling thread's current device for the scope and restores the caller's.
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) HIP_OK(hipSetDevice(dev));
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
};

class EnginePool {
 public:
  static constexpr int kMaxDev = 64;

  int devices() {
    std::call_once(once_, [&] {
      int n = 0;
      ndev_ = hipGetDeviceCount(&n) == hipSuccess ? std::min(n, kMaxDev) : 0;
      const char* c = getenv("BZG_ENGINES_PER_DEVICE");
      cap_ = c ? std::max(1, atoi(c)) : 4;
    });
    return ndev_;
  }

  // A free engine of device `dev` (created on demand up to the per-device cap, else waits).
  Engine* acquire(int dev) {
    if (dev < 0 || dev >= devices()) throw HipFailure(hipErrorInvalidDevice);
    std::unique_lock<std::mutex> g(mu_);
    for (;;) {
      if (!idle_[dev].empty()) {
        Engine* e = idle_[dev].back();
        idle_[dev].pop_back();
        return e;
      }
      if (count_[dev] < cap_) {
        count_[dev]++;
        g.unlock();
        try {
          DeviceScope ds(dev);
          return new Engine(dev);  // never destroyed: device teardown order at exit is unsafe
        } catch (...) {
          g.lock();
          count_[dev]--;
          cv_.notify_all();
          throw;
        }
      }
      cv_.wait(g);
    }
  }

  // Engines for every entry of devs (repeats allowed), taken together under one lock so that
  // concurrent multi-engine calls cannot deadlock holding part of their sets.
  std::vector<Engine*> acquire_set(const std::vector<int>& devs) {
    for (int d : devs)
      if (d < 0 || d >= devices()) throw HipFailure(hipErrorInvalidDevice);
    std::vector<int> want(kMaxDev, 0);
    for (int d : devs) want[d]++;
    for (int d = 0; d < kMaxDev; d++)
      if (want[d] > cap_) throw HipFailure(hipErrorInvalidValue);
    std::unique_lock<std::mutex> g(mu_);
    cv_.wait(g, [&] {
      for (int d = 0; d < kMaxDev; d++)
        if (want[d] && (int)idle_[d].size() + (cap_ - count_[d]) < want[d]) return false;
      return true;
    });
    std::vector<Engine*> out;
    std::vector<int> fresh;
    for (int d : devs) {
      if (!idle_[d].empty()) {
        out.push_back(idle_[d].back());
        idle_[d].pop_back();
      } else {
        count_[d]++;
        out.push_back(nullptr);
        fresh.push_back((int)out.size() - 1);
      }
    }
    g.unlock();
    try {
      for (int i : fresh) {
        DeviceScope ds(devs[i]);
        out[i] = new Engine(devs[i]);
      }
    } catch (...) {
      g.lock();
      for (size_t i = 0; i < out.size(); i++) {
        if (out[i]) idle_[out[i]->device].push_back(out[i]);
      }
      for (int i : fresh)
        if (!out[i]) count_[devs[i]]--;
      cv_.notify_all();
      throw;
    }
    return out;
  }

  void release(Engine* e) {
    {
      std::lock_guard<std::mutex> g(mu_);
      idle_[e->device].push_back(e);
    }
    cv_.notify_all();
  }

  // Frees the device memory of every idle engine (engines in use keep theirs).
  void release_idle_memory() {
    std::lock_guard<std::mutex> g(mu_);
    for (int d = 0; d < ndev_; d++)
      for (Engine* e : idle_[d]) {
        try {  // a C entry point calls this: nothing may escape
          DeviceScope ds(e->device);
          (void)hipStreamSynchronize(e->stream);
          for (auto x : e->sstream) (void)hipStreamSynchronize(x);
          e->release_idle();
        } catch (...) {
        }
      }
  }

 private:
  std::once_flag once_;
  int ndev_ = 0, cap_ = 4;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Engine*> idle_[kMaxDev];
  int count_[kMaxDev] = {};
};

static EnginePool& pool() {
  static EnginePool* p = new EnginePool();
  return *p;
}

// One engine of a device for the duration of a call, with the device made current.
struct Lease {
  DeviceScope ds;  // first: if switching the device throws, no engine has been taken yet
  Engine* e;
  explicit Lease(int dev) : ds(dev), e(pool().acquire(dev)) {}
  ~Lease() {
    e->own_streams();
    pool().release(e);
  }
  Engine* operator->() const { return e; }
  Lease(const Lease&) = delete;
  Lease& operator=(const Lease&) = delete;
};

// The calling thread's current HIP device (device pointers handed to the engine live there).
static int current_device() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) d = 0;
  return d;
}

// Device errors to bzlib codes: device allocation failure -> BZ_MEM_ERROR, a short caller
// output buffer -> BZ_OUTBUFF_FULL, anything else on the device -> BZ_CONFIG_ERROR.
template <typename F>
static int guarded(F&& f) {
  try {
    return f();
  } catch (const OutBuffFull&) {
    return BZ_OUTBUFF_FULL;
  } catch (const HipFailure& x) {
    return x.err == hipErrorOutOfMemory ? BZ_MEM_ERROR : BZ_CONFIG_ERROR;
  } catch (const CopyRankFailure&) {
    return BZ_CONFIG_ERROR;
  } catch (const std::bad_alloc&) {
    return BZ_MEM_ERROR;
  }
}

static std::mutex g_stats_mu;
static bzg_stats g_last{};
static void publish_stats(const bzg_stats& s) {
  std::lock_guard<std::mutex> g(g_stats_mu);
  g_last = s;
}

// State of the sharded-stream chunk map (bzg_seg_map / bzg_seg_walk): one per process, since a
// rank drives one region at a time; kept on its own engine so the walk finds the map.
struct SegState {
  std::mutex mu;
  Engine* e = nullptr;          // the engine of the current region's device
  std::vector<Engine*> by_dev;  // one per device, created on first use, kept for the process
  const uint8_t* in = nullptr;
  uint64_t n = 0;
  int level = 0;
  hipStream_t stream = nullptr;
};
static SegState& seg_state() {
  static SegState* s = new SegState();
  return *s;
}

// ---------------------------------------------------------------- several devices, one stream
// One .bz2 stream over several devices inside one process (bzg_compress_host with BZG_NGPUS
// > 1): the drop-in's callers (the CLI, BZ2_bzBuffToBuffCompress users) live in one process,
// so the node's GPUs are driven from here rather than from one process per GPU.  The steps
// are those of bzip2_amd/shard.py, in C++:
//  1. every device maps the RLE1 chunks of its shard of the input (in parallel);
//  2. the block cuts are walked shard after shard (bzlib.c:211-315: a block ends once it
//     holds >= nblockMAX RLE1 bytes; the pending run opens the next block; the stream's last
//     byte never opens one), the run crossing a shard start settled by arithmetic;
//  3. a block belongs to the device whose shard holds its first byte; every device compresses
//     its range of blocks (in parallel) as a flushed segment without trailer, the first range
//     with the stream header;
//  4. each device shifts its bits to the range's bit offset mod 8 and they are copied behind
//     each other into the caller's buffer (the shared boundary bytes OR-ed), then the combined
//     CRC (combined = rotl(combined, blocks_d) ^ crc_d, compress.c:826-828) and the trailer.
// The output is byte-identical to the single-device stream (the cuts do not depend on the
// sharding).  BZG_DEVICES="0,0,0" runs the same path with several engines on one device.
namespace {

__global__ void k_shift_bits(const uint8_t* __restrict__ in, uint64_t nbits, uint32_t sh, uint8_t* __restrict__ out) {
  // out = the first nbits bits of `in` moved sh bits later (0 <= sh < 8), trailing bits zero
  const uint64_t nbytes = (nbits + sh + 7) / 8, nin = (nbits + 7) / 8;
  const uint32_t tail = (uint32_t)(nbits & 7);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes; i += (uint64_t)gridDim.x * blockDim.x) {
    auto byte_at = [&](uint64_t j) -> uint32_t {
      if (j >= nin) return 0u;
      uint32_t v = in[j];
      if (j + 1 == nin && tail) v &= (0xffu << (8 - tail)) & 0xffu;
      return v;
    };
    const uint32_t cur = byte_at(i), prev = i ? byte_at(i - 1) : 0u;
    out[i] = (uint8_t)(((cur >> sh) | (prev << (8 - sh))) & 0xffu);
  }
}

struct Shard {
  int dev;
  uint64_t s, e;         // input shard [s, e)
  uint64_t p;            // first run start inside the shard (relative)
  Engine* eng = nullptr;
  uint8_t* d_shard = nullptr;
  std::vector<uint64_t> cuts;  // global block starts inside the shard
  uint64_t lo = 0, hi = 0;     // owned range
  uint64_t nbits = 0;
  uint32_t nblocks = 0, crc = 0;
  uint8_t* d_bits = nullptr;   // shifted bits
  uint64_t nshift = 0;
  bzg_stats stats{};
};

inline uint32_t chunk_size(uint64_t len) { return len < 4 ? (uint32_t)len : 5u; }

// first j >= 1 with x[j] != x[j - 1] (or len)
uint64_t first_run_start(const uint8_t* x, uint64_t len) {
  uint64_t j = 1;
  while (j < len && x[j] == x[j - 1]) j++;
  return j;
}

// the chunks of a run piece [t, x) of equal bytes whose first chunk starts at t (chunks every
// 255 bytes, 5 RLE1 bytes each): cuts where the block fills (never at the stream's last byte)
void extend_run(uint64_t& t, uint32_t& fill, uint64_t x, uint32_t mx, std::vector<uint64_t>& cuts, uint64_t last_pos) {
  uint64_t q = (x - t - 1) / 255;
  while (q > 0) {
    const uint64_t need = fill >= mx ? 1 : std::max<uint64_t>(1, (mx - fill + 4) / 5);
    if (need <= q) {
      t += 255 * need;
      q -= need;
      if (t != last_pos) {
        cuts.push_back(t);
        fill = 0;
      } else {
        fill += (uint32_t)(5 * need);
      }
    } else {
      t += 255 * q;
      fill += (uint32_t)(5 * q);
      q = 0;
    }
  }
}

struct ChainMsg {
  bool valid = false;
  uint64_t t = 0;      // start of the open chunk
  uint32_t fill = 0;   // block fill before it
  uint8_t byte = 0;
  uint64_t covered = 0;
};

}  // namespace

static int compress_host_multi(const uint8_t* src, uint64_t n, int level, uint8_t* dst, uint64_t dst_cap,
                               uint64_t* dst_len, const std::vector<int>& devs) {
  const uint32_t mx = 100000u * (uint32_t)level - 19u;
  const size_t N = devs.size();
  std::vector<Shard> sh(N);
  for (size_t d = 0; d < N; d++) {
    sh[d].dev = devs[d];
    sh[d].s = n * d / N;
    sh[d].e = n * (d + 1) / N;
  }
  // engines for the whole call (every engine keeps its chunk map between the steps), taken as
  // one set and returned to the pool on every exit path
  struct SetLease {
    std::vector<Engine*> e;
    ~SetLease() {
      for (Engine* x : e) pool().release(x);
    }
  } lease{pool().acquire_set(devs)};
  for (size_t d = 0; d < N; d++) sh[d].eng = lease.e[d];
  auto parallel = [&](auto&& fn) {
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> err(N);
    for (size_t d = 0; d < N; d++)
      th.emplace_back([&, d] {
        try {
          DeviceScope ds(sh[d].dev);
          fn(sh[d]);
        } catch (...) {
          err[d] = std::current_exception();
        }
      });
    for (auto& t : th) t.join();
    for (auto& e : err)
      if (e) std::rethrow_exception(e);
  };
  // 1. shards in device memory and their chunk maps
  parallel([&](Shard& S) {
    const uint64_t len = S.e - S.s;
    S.p = first_run_start(src + S.s, len);
    S.d_shard = S.eng->ws.u8("mg_shard", len + 64);
    HIP_OK(hipMemcpyAsync(S.d_shard, src + S.s, len, hipMemcpyHostToDevice, S.eng->stream));
    if (S.p < len) seg_map_stage(S.eng->ws, S.d_shard + S.p, len - S.p, S.eng->stream);
    HIP_OK(hipStreamSynchronize(S.eng->stream));
  });
  // 2. the cut chain, shard after shard
  const uint64_t last_pos = n - 1;
  ChainMsg msg;
  for (size_t d = 0; d < N; d++) {
    Shard& S = sh[d];
    DeviceScope ds(S.dev);
    const uint64_t len = S.e - S.s;
    const bool final = d + 1 == N;
    const uint8_t d0 = src[S.s], dlast = src[S.e - 1];
    uint64_t t;
    uint32_t fill;
    if (!msg.valid) {
      t = S.s;
      fill = 0;
    } else {
      t = msg.t;
      fill = msg.fill;
      if (msg.byte != d0 || msg.covered >= 255) {  // the open chunk ends at the shard start
        fill += chunk_size(msg.covered);
        t = S.s;
        if (fill >= mx && S.s != last_pos) {
          S.cuts.push_back(S.s);
          fill = 0;
        }
      }
    }
    const uint64_t x = S.s + S.p;  // [t, x) is one run piece of byte d0
    extend_run(t, fill, x, mx, S.cuts, last_pos);
    msg = ChainMsg{};
    if (S.p == len) {  // the whole shard is one run piece
      if (!final) msg = ChainMsg{true, t, fill, d0, S.e - t};
      continue;
    }
    fill += chunk_size(x - t);  // the run ends at x, a run start
    if (x == last_pos) continue;  // the stream's last byte joins the open block
    if (fill >= mx) {
      S.cuts.push_back(x);
      fill = 0;
    }
    std::vector<uint64_t> rc;
    uint64_t lc = 0;
    uint32_t lf = fill;
    seg_walk_stage(S.eng->ws, S.d_shard + S.p, len - S.p, level, fill, final, rc, lc, lf, S.eng->stream);
    for (uint64_t c : rc) S.cuts.push_back(x + c);
    if (!final) msg = ChainMsg{true, x + lc, lf, dlast, S.e - (x + lc)};
  }
  // 3. owned ranges: from the first block start in the shard to the next owner's
  {
    std::vector<uint64_t> first(N, UINT64_MAX);
    for (size_t d = 0; d < N; d++) {
      if (d == 0) first[d] = 0;
      else if (!sh[d].cuts.empty()) first[d] = sh[d].cuts.front();
    }
    // a cut made by shard d's walk lies inside shard d, except the arithmetic ones of a run
    // crossing into later shards: assign every cut to the shard holding it
    std::vector<uint64_t> all;
    for (auto& S : sh) all.insert(all.end(), S.cuts.begin(), S.cuts.end());
    std::sort(all.begin(), all.end());
    for (size_t d = 1; d < N; d++) {
      auto it = std::lower_bound(all.begin(), all.end(), sh[d].s);
      first[d] = (it != all.end() && *it < sh[d].e) ? *it : UINT64_MAX;
    }
    for (size_t d = 0; d < N; d++) {
      if (first[d] == UINT64_MAX) continue;
      uint64_t nx = n;
      for (size_t j = d + 1; j < N; j++)
        if (first[j] != UINT64_MAX) {
          nx = first[j];
          break;
        }
      sh[d].lo = first[d];
      sh[d].hi = nx;
    }
  }
  // 4. compress the ranges, shift the bits to their byte offsets on the device.  A range is
  // built from the shards already on the devices: in place when it lies in the own shard,
  // else the own part plus the tail of later shards copied device to device (xGMI peer copies
  // between GPUs) -- the input crosses PCIe once.
  parallel([&](Shard& S) {
    if (S.hi <= S.lo) return;
    Engine& E = *S.eng;
    const uint64_t len = S.hi - S.lo;
    const uint8_t* din = S.d_shard + (S.lo - S.s);
    if (S.hi > S.e) {
      uint8_t* buf = E.ws.u8("mg_in", len + 64);
      HIP_OK(hipMemcpyAsync(buf, S.d_shard + (S.lo - S.s), S.e - S.lo, hipMemcpyDeviceToDevice, E.stream));
      for (size_t j = (size_t)(&S - sh.data()) + 1; j < N && sh[j].s < S.hi; j++) {
        const uint64_t a = sh[j].s, b = std::min(S.hi, sh[j].e);
        HIP_OK(hipMemcpyPeerAsync(buf + (a - S.lo), S.dev, sh[j].d_shard, sh[j].dev, b - a, E.stream));
      }
      din = buf;
    }
    const uint64_t cap = bzg_bound(len) + 64;
    uint8_t* dout = E.ws.u8("mg_out", cap);
    bzg_stream_state st;
    bzg_stream_init(&st, level);
    st.header_done = S.lo == 0 ? 0 : 1;
    const unsigned flags = BZG_FLAG_END_SEGMENT | (S.hi == n ? BZG_FLAG_TAIL_MERGE : 0u);
    uint64_t ob = 0, cons = 0;
    E.compress(din, len, flags, &st, dout, cap, &ob, &cons, E.stream, S.stats);
    S.nbits = 8 * ob + st.carry_bits;
    if (st.carry_bits) {  // the unfinished last byte (not part of the ob whole bytes)
      HIP_OK(hipMemcpyAsync(dout + ob, &st.carry_byte, 1, hipMemcpyHostToDevice, E.stream));
      HIP_OK(hipStreamSynchronize(E.stream));
    }
    S.nblocks = st.blocks_done;
    S.crc = st.combined_crc;
  });
  uint64_t total_bits = 0;
  std::vector<uint64_t> off(N);
  for (size_t d = 0; d < N; d++) {
    off[d] = total_bits;
    total_bits += sh[d].nbits;
  }
  const uint64_t out_len = (total_bits + 80 + 7) / 8;
  if (out_len > dst_cap) return BZ_OUTBUFF_FULL;
  // 5. gather on the first device: every range's shifted bytes but its first (shared with the
  // previous range's last byte, OR-ed on the host) are peer-copied to their byte offset, then
  // one copy to the caller's buffer
  uint8_t* gat = nullptr;
  {
    Engine& E0 = *sh[0].eng;
    DeviceScope ds0(sh[0].dev);
    gat = E0.ws.u8("mg_gather", out_len + 64);
    HIP_OK(hipMemsetAsync(gat, 0, out_len, E0.stream));
    HIP_OK(hipStreamSynchronize(E0.stream));
  }
  std::vector<uint8_t> head(N, 0);
  parallel([&](Shard& S) {
    const size_t d = &S - sh.data();
    if (S.nbits == 0) return;
    Engine& E = *S.eng;
    const uint32_t s8 = (uint32_t)(off[d] & 7);
    const uint64_t nb = (S.nbits + s8 + 7) / 8;
    uint8_t* dout = E.ws.u8("mg_out", 1);  // same buffer (already large enough)
    uint8_t* dsh = E.ws.u8("mg_shift", nb + 64);
    k_shift_bits<<<(unsigned)std::min<uint64_t>(ceil_div64(nb, 256), 65536), 256, 0, E.stream>>>(dout, S.nbits, s8,
                                                                                               dsh);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(&head[d], dsh, 1, hipMemcpyDeviceToHost, E.stream));
    if (nb > 1) HIP_OK(hipMemcpyPeerAsync(gat + off[d] / 8 + 1, sh[0].dev, dsh + 1, S.dev, nb - 1, E.stream));
    HIP_OK(hipStreamSynchronize(E.stream));
  });
  {
    Engine& E0 = *sh[0].eng;
    DeviceScope ds0(sh[0].dev);
    HIP_OK(hipMemcpyAsync(dst, gat, out_len, hipMemcpyDeviceToHost, E0.stream));
    HIP_OK(hipStreamSynchronize(E0.stream));
  }
  uint32_t comb = 0;
  bzg_stats acc{};
  for (size_t d = 0; d < N; d++) {
    if (sh[d].nbits) dst[off[d] / 8] |= head[d];
    const uint32_t k = sh[d].nblocks % 32;
    if (k) comb = (comb << k) | (comb >> (32 - k));
    comb ^= sh[d].crc;
    acc.total_ms = std::max(acc.total_ms, sh[d].stats.total_ms);
    acc.nblocks += sh[d].stats.nblocks;
    acc.rle_bytes += sh[d].stats.rle_bytes;
    acc.mtf_symbols += sh[d].stats.mtf_symbols;
  }
  publish_stats(acc);
  // trailer: 0x177245385090 and the combined CRC at bit total_bits, zero padded
  {
    const uint64_t tr_hi = 0x177245385090ull;
    uint64_t bit = total_bits;
    auto put = [&](uint64_t v, int nbits) {
      for (int i = nbits - 1; i >= 0; i--, bit++)
        if ((v >> i) & 1u) dst[bit >> 3] |= (uint8_t)(0x80u >> (bit & 7));
    };
    put(tr_hi, 48);
    put(comb, 32);
  }
  *dst_len = out_len;
  return BZ_OK;
}

// Devices of the multi-device path: BZG_DEVICES (a list, repeats allowed) or the first
// BZG_NGPUS devices; empty when the single-device path applies.
static std::vector<int> multi_devices(uint64_t n) {
  std::vector<int> devs;
  const char* list = getenv("BZG_DEVICES");
  const char* ng = getenv("BZG_NGPUS");
  const int ndev = pool().devices();
  if (list && *list) {
    for (const char* p = list; *p;) {
      char* end = nullptr;
      const long v = strtol(p, &end, 10);
      if (end == p) break;
      if (v >= 0 && v < ndev) devs.push_back((int)v);
      p = *end ? end + 1 : end;
    }
  } else if (ng) {
    const int k = std::min(atoi(ng), ndev);
    for (int d = 0; d < k; d++) devs.push_back(d);
  }
  // a device listed more often than it has engines would block the call: clamp the repeats
  {
    const char* c = getenv("BZG_ENGINES_PER_DEVICE");
    const int cap = c ? std::max(1, atoi(c)) : 4;
    std::vector<int> seen(std::max(ndev, 1), 0), kept;
    for (int d : devs)
      if (seen[d]++ < cap) kept.push_back(d);
    devs.swap(kept);
  }
  // worth it only for inputs of several blocks per device; shards within one batch
  if (devs.size() < 2 || n < (uint64_t)devs.size() * 4000000ull || n / devs.size() + 1 > kMaxBatchLimit) devs.clear();
  return devs;
}

}  // namespace bzg

using namespace bzg;

extern "C" {

void bzg_stream_init(bzg_stream_state* st, int level) {
  std::memset(st, 0, sizeof(*st));
  st->level = (uint8_t)level;
}

uint64_t bzg_bound(uint64_t n) { return n + n / 50 + (n / 100000 + 2) * 64 + 4096; }

int bzg_device_ok(void) {
  if (pool().devices() <= 0) return 0;
  const int rc = guarded([&] {
    Lease L(current_device());
    return BZ_OK;
  });
  return rc == BZ_OK ? 1 : 0;
}

int bzg_compress_device(const void* d_in, uint64_t n, unsigned flags, bzg_stream_state* st, void* d_out,
                        uint64_t out_cap, uint64_t* out_bytes, uint64_t* consumed, void* stream) {
  if (!st || !out_bytes || !consumed || st->level < 1 || st->level > 9 || (n && !d_in) || !d_out)
    return BZ_PARAM_ERROR;
  if (pool().devices() <= 0) return BZ_CONFIG_ERROR;
  return guarded([&] {
    Lease L(current_device());
    hipStream_t s = stream ? (hipStream_t)stream : L->stream;
    bzg_stats last{};
    L->compress((const uint8_t*)d_in, n, flags, st, (uint8_t*)d_out, out_cap, out_bytes, consumed, s, last);
    publish_stats(last);
    return BZ_OK;
  });
}

int bzg_seg_map(const void* d_in, uint64_t n, int level, void* stream) {
  if (level < 1 || level > 9 || (n && !d_in) || n > kMaxBatchLimit) return BZ_PARAM_ERROR;
  if (pool().devices() <= 0) return BZ_CONFIG_ERROR;
  SegState& S = seg_state();
  std::lock_guard<std::mutex> g(S.mu);
  S.in = nullptr;
  return guarded([&] {
    const int dev = current_device();
    if (S.by_dev.size() <= (size_t)dev) S.by_dev.resize(dev + 1, nullptr);
    if (!S.by_dev[dev]) {
      DeviceScope ds(dev);
      S.by_dev[dev] = new Engine(dev);
    }
    S.e = S.by_dev[dev];
    DeviceScope ds(dev);
    hipStream_t s = stream ? (hipStream_t)stream : S.e->stream;
    S.e->ws.set_stream(s);
    seg_map_stage(S.e->ws, (const uint8_t*)d_in, n, s);
    S.in = (const uint8_t*)d_in;
    S.n = n;
    S.level = level;
    S.stream = s;
    return BZ_OK;
  });
}

int bzg_seg_walk(uint32_t fill_in, int final_region, uint64_t* cuts, uint32_t max_cuts, uint32_t* ncuts,
                 uint64_t* last_chunk, uint32_t* last_fill) {
  if (!ncuts || !last_chunk || !last_fill || (max_cuts && !cuts)) return BZ_PARAM_ERROR;
  SegState& S = seg_state();
  std::lock_guard<std::mutex> g(S.mu);
  if (!S.e || (!S.in && S.n)) return BZ_PARAM_ERROR;  // no successful bzg_seg_map
  if (fill_in >= 100000u * (uint32_t)S.level - 19u) return BZ_PARAM_ERROR;
  return guarded([&] {
    DeviceScope ds(S.e->device);
    std::vector<uint64_t> c;
    uint64_t lc = 0;
    uint32_t lf = fill_in;
    seg_walk_stage(S.e->ws, S.in, S.n, S.level, fill_in, final_region != 0, c, lc, lf, S.stream);
    if (c.size() > max_cuts) return BZ_OUTBUFF_FULL;
    for (size_t i = 0; i < c.size(); i++) cuts[i] = c[i];
    *ncuts = (uint32_t)c.size();
    *last_chunk = lc;
    *last_fill = lf;
    return BZ_OK;
  });
}

int bzg_find_magics(const void* d_in, uint64_t n, uint64_t* out, uint64_t cap, uint64_t* count, void* stream) {
  if ((n && !d_in) || !count || (cap && !out)) return BZ_PARAM_ERROR;
  if (pool().devices() <= 0) return BZ_CONFIG_ERROR;
  return guarded([&] {
    Lease L(current_device());
    hipStream_t s = stream ? (hipStream_t)stream : L->stream;
    std::vector<uint64_t> f;
    find_magics_stage((const uint8_t*)d_in, n, f, s);
    *count = f.size();
    for (uint64_t i = 0; i < f.size() && i < cap; i++) out[i] = f[i];
    return f.size() > cap ? BZ_OUTBUFF_FULL : BZ_OK;
  });
}

// Host buffers of large inputs: the input goes over in pieces, on the engine's copy stream from a
// copier thread, while the main thread compresses the pieces that have arrived as consecutive
// segments of one stream (a non-final segment emits its complete blocks and the rest is
// resubmitted with the next piece, exactly as bzg_compress_device cuts a large input into
// batches, so the bytes equal one call's); each segment's output goes back from a second thread
// while the next one is compressed.  The pieces are the batches of Engine::compress_pipelined,
// so a piece's back stage (MTF, tables, packing) runs beside the next piece's sorts.  Only the
// first piece's upload and the last piece's back stage and download are not overlapped.  A
// piece has a fixed cost (host synchronisations of the sort passes, narrow late passes; a
// 100 MB call takes 7.5 ms against 4.8 ms at the 1 GB rate), so pieces are few: from 640 MiB,
// 10% (its upload is the only wait), 30% and 40% (each upload is covered by the compression of
// the piece before, at ~53 GB/s) and a last 20% (short back stage and download); below that,
// a fifth and the rest (profiles/r06_h2h_plans.txt, r05_h2h_*.txt).
static constexpr uint64_t kPipeMin = 192ull << 20;  // smaller inputs: one upload, one call, one download
static constexpr uint64_t kPipeFirst = 96ull << 20;
static constexpr uint64_t kPipe4 = 640ull << 20;  // from here: four pieces

static std::vector<uint64_t> pipe_pieces(uint64_t n) {
  std::vector<uint64_t> b{0};
  if (const char* plan = getenv("BZG_H2H_PLAN")) {  // A/B knob: leading piece sizes in MB, "100,300"
    for (const char* q = plan; *q;) {
      char* e = nullptr;
      const unsigned long long mb = strtoull(q, &e, 10);
      if (e == q) break;
      if (mb && b.back() + (mb << 20) < n) b.push_back(b.back() + (mb << 20));
      q = *e ? e + 1 : e;
    }
    b.push_back(n);
    return b;
  }
  if (n >= kPipe4) {  // 10% + 30% + 40% + 20% (profiles/r06_h2h_plans.txt)
    for (uint64_t f : {1u, 4u, 8u}) b.push_back(n / 10 * f);
    b.push_back(n);
    return b;
  }
  uint64_t s = std::max<uint64_t>(kPipeFirst, n / 5);  // (n/4, n/8, 3 pieces: slower, profiles/r05_h2h_split.txt)
  while (n - b.back() > 4 * s) {
    b.push_back(b.back() + s);
    s *= 2;
  }
  b.push_back(n);
  return b;
}

static int host_call_pipelined(Engine* e, const uint8_t* src, uint64_t n, unsigned flags, bzg_stream_state* st,
                               uint8_t* dst, uint64_t dst_cap, uint64_t* dst_len, uint64_t* consumed) {
  const std::vector<uint64_t> b = pipe_pieces(n);
  const size_t J = b.size() - 1;
  const uint64_t cap = bzg_bound(n);
  uint8_t* din = e->ws.u8("host_in", n + 16);
  uint8_t* dout = e->ws.u8("host_out", cap);
  std::vector<hipEvent_t> ev_in(J, nullptr);
  for (auto& x : ev_in) HIP_OK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  std::mutex mu;
  std::condition_variable cv;
  size_t uploaded = 0;     // pieces whose copy is queued (ev_in recorded)
  bool up_failed = false;
  struct Down { uint64_t off, len; };
  std::vector<Down> downs;  // segment outputs to copy back, in order
  bool all_queued = false, down_failed = false;
  const int dev = e->device;
  // BZG_H2H_DEBUG: host times (ms since the call) of each piece's upload, compression and download
  static const bool dbg = getenv("BZG_H2H_DEBUG") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  std::thread up([&] {
    bool ok = hipSetDevice(dev) == hipSuccess;
    for (size_t j = 0; j < J && ok; j++) {
      ok = hipMemcpyAsync(din + b[j], src + b[j], b[j + 1] - b[j], hipMemcpyHostToDevice, e->cstream) == hipSuccess &&
           hipEventRecord(ev_in[j], e->cstream) == hipSuccess;
      if (dbg) {
        const double a = ms();
        (void)hipEventSynchronize(ev_in[j]);
        fprintf(stderr, "[bzg h2h] piece %zu (%llu B): upload queued %.2f done %.2f ms\n", j,
                (unsigned long long)(b[j + 1] - b[j]), a, ms());
      }
      std::lock_guard<std::mutex> g(mu);
      if (ok) uploaded = j + 1;
      else up_failed = true;
      cv.notify_all();
    }
  });
  std::thread down([&] {
    bool ok = hipSetDevice(dev) == hipSuccess;
    for (size_t i = 0;; i++) {
      Down d;
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return i < downs.size() || all_queued; });
        if (i >= downs.size()) break;
        d = downs[i];
      }
      if (ok && d.len) ok = hipMemcpy(dst + d.off, dout + d.off, d.len, hipMemcpyDeviceToHost) == hipSuccess;
      if (dbg) fprintf(stderr, "[bzg h2h] download %zu (%llu B) done %.2f ms\n", i, (unsigned long long)d.len, ms());
      if (!ok) {
        std::lock_guard<std::mutex> g(mu);
        down_failed = true;
      }
    }
  });
  auto finish_threads = [&] {
    {
      std::lock_guard<std::mutex> g(mu);
      all_queued = true;
    }
    cv.notify_all();
    up.join();
    down.join();
    for (auto& x : ev_in) (void)hipEventDestroy(x);
  };
  // The pieces are the batches of Engine::compress_pipelined: the front stage of a piece (its
  // RLE1 and sorts) waits for its upload and runs beside the previous piece's back stage; each
  // piece's coded bytes go to the download thread as soon as they are packed.
  Engine::PipeHooks hk;
  hk.ends.assign(b.begin() + 1, b.end());
  size_t waited = 0;  // pieces the caller's stream already waits for
  hk.wait_input = [&](uint64_t end) {
    while (waited < J && b[waited] < end) {
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return uploaded > waited || up_failed; });
        if (uploaded <= waited) throw HipFailure(hipErrorUnknown);
      }
      HIP_OK(hipStreamWaitEvent(e->stream, ev_in[waited], 0));
      if (dbg) fprintf(stderr, "[bzg h2h] piece %zu: compression may start %.2f ms\n", waited, ms());
      waited++;
    }
  };
  bool overflow = false;
  hk.on_output = [&](uint64_t off, uint64_t len) {
    if (dbg) fprintf(stderr, "[bzg h2h] coded [%llu, +%llu) ready %.2f ms\n", (unsigned long long)off,
                     (unsigned long long)len, ms());
    {
      std::lock_guard<std::mutex> g(mu);
      if (off + len > dst_cap) overflow = true;
      else downs.push_back(Down{off, len});
    }
    cv.notify_all();
  };
  uint64_t done_in = 0, done_out = 0;
  bzg_stats acc{};
  try {
    e->compress_pipelined(din, n, flags, st, dout, cap, &done_out, &done_in, e->stream, acc, &hk);
  } catch (...) {
    finish_threads();
    throw;
  }
  finish_threads();
  publish_stats(acc);
  if (overflow || done_out > dst_cap) return BZ_OUTBUFF_FULL;
  if (up_failed || down_failed) throw HipFailure(hipErrorUnknown);
  *dst_len = done_out;
  if (consumed) *consumed = done_in;
  return BZ_OK;
}

// Host buffers through one leased engine: staging, compression and copy-out all happen under
// the lease, so concurrent callers never share staging buffers.
static int host_call(const void* src, uint64_t n, unsigned flags, bzg_stream_state* st, void* dst, uint64_t dst_cap,
                     uint64_t* dst_len, uint64_t* consumed) {
  if (pool().devices() <= 0) return BZ_CONFIG_ERROR;
  return guarded([&] {
    Lease L(current_device());
    if (n >= kPipeMin && (flags & BZG_FLAG_END_SEGMENT))
      return host_call_pipelined(L.e, (const uint8_t*)src, n, flags, st, (uint8_t*)dst, dst_cap, dst_len, consumed);
    const uint64_t cap = bzg_bound(n);
    uint8_t* din = L->ws.u8("host_in", n + 16);
    uint8_t* dout = L->ws.u8("host_out", cap);
    if (n) HIP_OK(hipMemcpyAsync(din, src, n, hipMemcpyHostToDevice, L->stream));
    uint64_t ob = 0, cons = 0;
    bzg_stats last{};
    L->compress(din, n, flags, st, dout, cap, &ob, &cons, L->stream, last);
    publish_stats(last);
    if (ob > dst_cap) return BZ_OUTBUFF_FULL;
    if (ob) HIP_OK(hipMemcpyAsync(dst, dout, ob, hipMemcpyDeviceToHost, L->stream));
    HIP_OK(hipStreamSynchronize(L->stream));
    *dst_len = ob;
    if (consumed) *consumed = cons;
    return BZ_OK;
  });
}

int bzg_compress_host(const void* src, uint64_t n, int level, void* dst, uint64_t dst_cap, uint64_t* dst_len) {
  if (level < 1 || level > 9 || (n && !src) || !dst || !dst_len) return BZ_PARAM_ERROR;
  if (pool().devices() > 0) {
    const std::vector<int> devs = multi_devices(n);
    if (!devs.empty())
      return guarded([&] {
        return compress_host_multi((const uint8_t*)src, n, level, (uint8_t*)dst, dst_cap, dst_len, devs);
      });
  }
  bzg_stream_state st;
  bzg_stream_init(&st, level);
  const unsigned flags = BZG_FLAG_END_SEGMENT | BZG_FLAG_TRAILER | (n ? BZG_FLAG_TAIL_MERGE : 0u);
  return host_call(src, n, flags, &st, dst, dst_cap, dst_len, nullptr);
}

int bzg_compress_host_stream(const void* src, uint64_t n, unsigned flags, bzg_stream_state* st, void* dst,
                             uint64_t dst_cap, uint64_t* dst_len, uint64_t* consumed) {
  if (!st || !dst || !dst_len || !consumed || (n && !src) || st->level < 1 || st->level > 9) return BZ_PARAM_ERROR;
  // the stream state advances only if the call succeeds
  bzg_stream_state work = *st;
  const int rc = host_call(src, n, flags, &work, dst, dst_cap, dst_len, consumed);
  if (rc == BZ_OK) *st = work;
  return rc;
}

// ---------------------------------------------------------------- decompression
static std::mutex g_dstats_mu;
static bzg_decode_stats g_dlast{};

static void publish_decode_stats(const DecodeStats& d) {
  std::lock_guard<std::mutex> g(g_dstats_mu);
  g_dlast.total_ms = d.total_ms;
  g_dlast.blocks = d.blocks;
  g_dlast.candidates = d.candidates;
  g_dlast.out_bytes = d.out_bytes;
}

int bzg_decompress_device(const void* d_in, uint64_t n, void* d_out, uint64_t out_cap, uint64_t* out_len, void* stream) {
  if ((n && !d_in) || (out_cap && !d_out) || !out_len) return BZ_PARAM_ERROR;
  if (pool().devices() <= 0) return BZ_CONFIG_ERROR;
  return guarded([&] {
    Lease L(current_device());
    hipStream_t s = stream ? (hipStream_t)stream : L->stream;
    DecodeStats ds;
    const int rc = decode_stage(L->ws, (const uint8_t*)d_in, n, (uint8_t*)d_out, out_cap, out_len, &ds, s);
    publish_decode_stats(ds);
    return rc;
  });
}

int bzg_decompress_host(const void* src, uint64_t n, void* dst, uint64_t dst_cap, uint64_t* dst_len) {
  if ((n && !src) || (dst_cap && !dst) || !dst_len) return BZ_PARAM_ERROR;
  if (pool().devices() <= 0) return BZ_CONFIG_ERROR;
  return guarded([&] {
    Lease L(current_device());
    uint8_t* din = L->ws.u8("dhost_in", n + 16);
    uint8_t* dout = L->ws.u8("dhost_out", dst_cap + 16);
    if (n) HIP_OK(hipMemcpyAsync(din, src, n, hipMemcpyHostToDevice, L->stream));
    DecodeStats ds;
    uint64_t got = 0;
    L->ws.set_stream(L->stream);
    const int rc = decode_stage(L->ws, din, n, dout, dst_cap, &got, &ds, L->stream);
    if (got) HIP_OK(hipMemcpyAsync(dst, dout, got, hipMemcpyDeviceToHost, L->stream));
    HIP_OK(hipStreamSynchronize(L->stream));
    *dst_len = got;
    publish_decode_stats(ds);
    return rc;
  });
}

void bzg_last_decode_stats(bzg_decode_stats* out) {
  std::lock_guard<std::mutex> g(g_dstats_mu);
  if (out) *out = g_dlast;
}

void bzg_last_stats(bzg_stats* out) {
  std::lock_guard<std::mutex> g(g_stats_mu);
  if (out) *out = g_last;
}

void bzg_release(void) {
  bzg::copyrank_memo_clear();
  if (pool().devices() <= 0) return;
  pool().release_idle_memory();
  SegState& S = seg_state();  // the chunk-map engines' workspaces too
  std::lock_guard<std::mutex> g(S.mu);
  for (Engine* e : S.by_dev)
    if (e) try {
        DeviceScope ds(e->device);
        (void)hipStreamSynchronize(e->stream);
        e->release_idle();
      } catch (...) {
      }
  S.in = nullptr;
  S.n = 0;
}

int32_t bzg_copy_rank_closed_form(const uint8_t* root, int32_t p, int32_t k) {
  if (!root || p < 2 || k < 2) return -1;
  try {
    const int32_t r = copy_rank_single(root, p, k);
    return r >= 0 ? r : copy_rank_distinct(root, p, k);
  } catch (...) {
    return -1;
  }
}

int32_t bzg_periodic_origptr(const uint8_t* block, int32_t n) {
  if (!block || n <= 0) return -1;
  try {
    const int32_t p = primitive_period(block, n);
    if (p == n) return -1;  // not periodic: the sort's rank is the origPtr
    if (p == 1) return 0;   // one symbol: no B* rotation
    const int32_t k = n / p;
    int32_t r = copy_rank_single(block, p, k);  // the device's closed forms first (origptr.hip)
    if (r < 0) r = copy_rank_distinct(block, p, k);
    if (r < 0) r = copy_rank(block, p, k);
    return root_rotation_rank(block, p) * k + r;
  } catch (const CopyRankFailure&) {
    return -1;
  } catch (const std::bad_alloc&) {
    return -1;
  }
}

// ---------------------------------------------------------------- per-stage entry points
// The stage hooks copy on the engine's stream, where its workspace buffers are allocated and
// freed (hipMallocAsync / hipFreeAsync), and wait for the copy.
static void stage_copy(Engine& e, void* dst, const void* src, size_t n, hipMemcpyKind kind) {
  HIP_OK(hipMemcpyAsync(dst, src, n, kind, e.stream));
  HIP_OK(hipStreamSynchronize(e.stream));
}
int bzg_stage_rle1(const void* src, uint64_t n, int level, int tail_merge, uint8_t* blocks, uint64_t blocks_cap,
                   uint32_t* offsets, uint32_t* crcs, uint32_t* nblocks, uint32_t max_blocks) {
  if (pool().devices() <= 0) return BZ_CONFIG_ERROR;
  Lease* lp = nullptr;
  try {
    lp = new Lease(current_device());
  } catch (const HipFailure&) {
    return BZ_CONFIG_ERROR;
  }
  std::unique_ptr<Lease> lease(lp);
  Engine& e = *lease->e;
  try {
    uint8_t* din = e.ws.u8("stage_in", n + 16);
    stage_copy(e, din, src, n, hipMemcpyHostToDevice);
    Rle1Result r;
    rle1_stage(e.ws, din, n, level, true, tail_merge != 0, r, e.stream);
    HIP_OK(hipStreamSynchronize(e.stream));
    if (r.nblocks > max_blocks) return BZ_OUTBUFF_FULL;
    *nblocks = r.nblocks;
    if (r.nblocks == 0) {
      offsets[0] = 0;
      return BZ_OK;
    }
    stage_copy(e, offsets, r.boff, 4 * (r.nblocks + 1), hipMemcpyDeviceToHost);
    if (offsets[r.nblocks] > blocks_cap) return BZ_OUTBUFF_FULL;
    stage_copy(e, blocks, r.blk, offsets[r.nblocks], hipMemcpyDeviceToHost);
    stage_copy(e, crcs, r.bcrc, 4 * r.nblocks, hipMemcpyDeviceToHost);
    return BZ_OK;
  } catch (const HipFailure&) {
    return BZ_CONFIG_ERROR;
  }
}

int bzg_stage_bwt(const uint8_t* blocks, const uint32_t* offsets, uint32_t nb, uint8_t* bwt_out, int32_t* origptr) {
  if (pool().devices() <= 0) return BZ_CONFIG_ERROR;
  Lease* lp = nullptr;
  try {
    lp = new Lease(current_device());
  } catch (const HipFailure&) {
    return BZ_CONFIG_ERROR;
  }
  std::unique_ptr<Lease> lease(lp);
  Engine& e = *lease->e;
  try {
    if (nb == 0) return BZ_OK;
    const uint32_t total = offsets[nb];
    Rle1Result r;
    r.nblocks = nb;
    r.blk = e.ws.u8("blk", total + 64);
    r.boff = e.ws.u32("boff", nb + 2);
    stage_copy(e, r.blk, blocks, total, hipMemcpyHostToDevice);
    stage_copy(e, r.boff, offsets, 4 * (nb + 1), hipMemcpyHostToDevice);
    block_info_stage(e.ws, r, e.stream);
    std::vector<uint32_t> hboff(offsets, offsets + nb + 1), hper(nb), hbq(nb), hqp(nb);
    HIP_OK(hipMemcpyAsync(hper.data(), r.period, 4 * nb, hipMemcpyDeviceToHost, e.stream));
    HIP_OK(hipMemcpyAsync(hbq.data(), r.bq, 4 * nb, hipMemcpyDeviceToHost, e.stream));
    HIP_OK(hipMemcpyAsync(hqp.data(), r.qper, 4 * nb, hipMemcpyDeviceToHost, e.stream));
    HIP_OK(hipStreamSynchronize(e.stream));
    uint8_t* bwt = e.ws.u8("bwt", total + 16);
    uint32_t* rank0 = e.ws.u32("rank0", nb + 2);
    uint32_t* d_orig = e.ws.u32("origptr", nb + 2);
    CopyRankJob a5;
    copyrank_begin(e.ws, r, hboff, hper, hbq, a5, e.stream);
    bwt_stage(e.ws, r, hboff, hper, bwt, rank0, nullptr, e.stream, hqp.data());
    copyrank_finish(e.ws, r, rank0, d_orig, a5, e.stream);
    HIP_OK(hipMemcpyAsync(origptr, d_orig, 4 * nb, hipMemcpyDeviceToHost, e.stream));
    HIP_OK(hipStreamSynchronize(e.stream));
    copyrank_check(a5);
    stage_copy(e, bwt_out, bwt, total, hipMemcpyDeviceToHost);
    return BZ_OK;
  } catch (const HipFailure&) {
    return BZ_CONFIG_ERROR;
  }
}

int bzg_stage_mtf(const uint8_t* bwt_in, const uint32_t* offsets, uint32_t nb, uint16_t* mtfv, uint64_t mtfv_cap,
                  uint32_t* mtf_offsets, uint32_t* nmtf, uint32_t* freq) {
  if (pool().devices() <= 0) return BZ_CONFIG_ERROR;
  Lease* lp = nullptr;
  try {
    lp = new Lease(current_device());
  } catch (const HipFailure&) {
    return BZ_CONFIG_ERROR;
  }
  std::unique_ptr<Lease> lease(lp);
  Engine& e = *lease->e;
  try {
    if (nb == 0) return BZ_OK;
    const uint32_t total = offsets[nb];
    Rle1Result r;
    r.nblocks = nb;
    r.blk = e.ws.u8("blk", total + 64);
    r.boff = e.ws.u32("boff", nb + 2);
    stage_copy(e, r.blk, bwt_in, total, hipMemcpyHostToDevice);
    stage_copy(e, r.boff, offsets, 4 * (nb + 1), hipMemcpyHostToDevice);
    block_info_stage(e.ws, r, e.stream);
    MtfResult m;
    mtf_stage(e.ws, r, r.blk, nb, total, m, e.stream);
    HIP_OK(hipStreamSynchronize(e.stream));
    stage_copy(e, mtf_offsets, m.mtf_off, 4 * (nb + 1), hipMemcpyDeviceToHost);
    stage_copy(e, nmtf, m.nmtf, 4 * nb, hipMemcpyDeviceToHost);
    stage_copy(e, freq, m.freq, 4 * (size_t)nb * kMaxAlpha, hipMemcpyDeviceToHost);
    if (mtf_offsets[nb] > mtfv_cap) return BZ_OUTBUFF_FULL;
    stage_copy(e, mtfv, m.mtfv, 2 * (size_t)mtf_offsets[nb], hipMemcpyDeviceToHost);
    return BZ_OK;
  } catch (const HipFailure&) {
    return BZ_CONFIG_ERROR;
  }
}

int bzg_stage_code_lengths(const uint32_t* freq, const int32_t* alpha, uint32_t ntables, int max_len,
                           uint8_t* lens) {
  if (pool().devices() <= 0) return BZ_CONFIG_ERROR;
  Lease* lp = nullptr;
  try {
    lp = new Lease(current_device());
  } catch (const HipFailure&) {
    return BZ_CONFIG_ERROR;
  }
  std::unique_ptr<Lease> lease(lp);
  Engine& e = *lease->e;
  if (ntables == 0) return BZ_OK;
  for (uint32_t t = 0; t < ntables; t++)
    if (alpha[t] < 2 || alpha[t] > kMaxAlpha) return BZ_PARAM_ERROR;
  if (max_len < 1 || max_len > 32) return BZ_PARAM_ERROR;
  try {
    const size_t nf = (size_t)ntables * kMaxAlpha;
    uint32_t* d_freq = e.ws.u32("test_freq", nf);
    int32_t* d_alpha = reinterpret_cast<int32_t*>(e.ws.u32("test_alpha", ntables));
    uint8_t* d_lens = e.ws.u8("test_lens", nf);
    stage_copy(e, d_freq, freq, 4 * nf, hipMemcpyHostToDevice);
    stage_copy(e, d_alpha, alpha, 4 * (size_t)ntables, hipMemcpyHostToDevice);
    code_lengths_test(e.ws, d_freq, d_alpha, ntables, max_len, d_lens, e.stream);
    HIP_OK(hipStreamSynchronize(e.stream));
    stage_copy(e, lens, d_lens, nf, hipMemcpyDeviceToHost);
    return BZ_OK;
  } catch (const HipFailure&) {
    return BZ_CONFIG_ERROR;
  }
}

}  // extern "C"
