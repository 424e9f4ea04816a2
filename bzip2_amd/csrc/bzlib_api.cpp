// bzlib_api.cpp -- the core stream exports of libbz2.def (reference libbz2.def:4-27) over the
// GPU engine; the stdio / zlib-style exports are in bzfile.cpp, decompression in decode.cpp.
//
// Compression keeps the reference's streaming contract (bzlib.c:144-474): BZ_RUN returns
// BZ_RUN_OK iff progress was made, BZ_FLUSH / BZ_FINISH move the stream into FLUSHING /
// FINISHING and must be repeated with an unchanged avail_in until BZ_RUN_OK / BZ_STREAM_END.
// Input is staged on the host and compressed by the device in batches; output may lag input
// (the concatenated bytes are what the reference emits for the same call pattern):
//   * RUN-mode bytes are staged; once the stage limit is reached the complete blocks among
//     them are compressed (RUN semantics: a full block is cut, bzlib.c:383-386).  The limit
//     starts at two blocks' worth, so a streaming caller sees output about as soon as the
//     reference would emit it, and doubles with every device batch up to kStageMax, where a
//     batch amortises its launch and synchronisation cost;
//   * FLUSH / FINISH compress everything staged as the end of a segment; the final length-1
//     run chunk joins a full block only when bytes arrived with the FLUSH/FINISH call
//     (bzlib.c:276-308).
#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/bzg.h"
#include "../../include/bzlib.h"
#include "decode.h"

namespace {

constexpr int kModeIdle = 1, kModeRunning = 2, kModeFlushing = 3, kModeFinishing = 4;
constexpr size_t kStageMax = 256u << 20;

void* default_alloc(void*, int items, int size) { return std::malloc((size_t)items * (size_t)size); }
void default_free(void*, void* p) { std::free(p); }

struct CState {
  bz_stream* strm;
  int level, verbosity;
  int mode;
  unsigned avail_in_expect;
  bool segment_done;
  bool tail_merge;
  size_t stage_limit;
  std::vector<uint8_t> staged;
  std::vector<uint8_t> out;
  size_t out_pos;
  bzg_stream_state st;
};

void add64(unsigned& lo, unsigned& hi, unsigned n) {
  const unsigned t = lo + n;
  if (t < lo) hi++;
  lo = t;
}

// Moves all of strm's input into staging.  Returns true if any byte was taken.
bool take_input(CState* s) {
  bz_stream* z = s->strm;
  if (z->avail_in == 0) return false;
  s->staged.insert(s->staged.end(), (uint8_t*)z->next_in, (uint8_t*)z->next_in + z->avail_in);
  add64(z->total_in_lo32, z->total_in_hi32, z->avail_in);
  z->next_in += z->avail_in;
  z->avail_in = 0;
  return true;
}

// Copies pending output to the caller.  Returns true if any byte moved.
bool drain(CState* s) {
  bz_stream* z = s->strm;
  size_t left = s->out.size() - s->out_pos;
  size_t cnt = left < z->avail_out ? left : z->avail_out;
  if (cnt == 0) return false;
  std::memcpy(z->next_out, s->out.data() + s->out_pos, cnt);
  z->next_out += cnt;
  z->avail_out -= (unsigned)cnt;
  add64(z->total_out_lo32, z->total_out_hi32, (unsigned)cnt);
  s->out_pos += cnt;
  if (s->out_pos == s->out.size()) {
    s->out.clear();
    s->out_pos = 0;
  }
  return true;
}

// Compresses the staged bytes.  end_segment: FLUSH/FINISH; trailer: FINISH.
int run_device(CState* s, bool end_segment, bool trailer) {
  unsigned flags = 0;
  if (end_segment) flags |= BZG_FLAG_END_SEGMENT;
  if (end_segment && s->tail_merge) flags |= BZG_FLAG_TAIL_MERGE;
  if (trailer) flags |= BZG_FLAG_TRAILER;
  const uint64_t n = s->staged.size();
  const uint64_t cap = bzg_bound(n);
  const size_t base = s->out.size();
  s->out.resize(base + cap);
  uint64_t got = 0, consumed = 0;
  int rc = bzg_compress_host_stream(s->staged.data(), n, flags, &s->st, s->out.data() + base, cap, &got, &consumed);
  if (rc != BZ_OK) {
    s->out.resize(base);
    return rc == BZ_OUTBUFF_FULL ? BZ_MEM_ERROR : rc;
  }
  s->out.resize(base + got);
  s->staged.erase(s->staged.begin(), s->staged.begin() + (std::ptrdiff_t)consumed);
  return BZ_OK;
}

}  // namespace

extern "C" {

int BZ2_bzCompressInit(bz_stream* strm, int blockSize100k, int verbosity, int workFactor) {
  if (strm == nullptr || blockSize100k < 1 || blockSize100k > 9 || workFactor < 0 || workFactor > 250)
    return BZ_PARAM_ERROR;
  if (!bzg_device_ok()) return BZ_CONFIG_ERROR;
  if (strm->bzalloc == nullptr) strm->bzalloc = default_alloc;
  if (strm->bzfree == nullptr) strm->bzfree = default_free;
  void* mem = strm->bzalloc(strm->opaque, (int)sizeof(CState), 1);
  if (mem == nullptr) return BZ_MEM_ERROR;
  CState* s = new (mem) CState();
  s->strm = strm;
  s->level = blockSize100k;
  s->verbosity = verbosity;
  s->mode = kModeRunning;
  s->avail_in_expect = 0;
  s->segment_done = false;
  s->tail_merge = false;
  s->stage_limit = 2 * (size_t)100000 * (size_t)blockSize100k + 64;
  s->out_pos = 0;
  bzg_stream_init(&s->st, blockSize100k);
  strm->state = s;
  strm->total_in_lo32 = strm->total_in_hi32 = 0;
  strm->total_out_lo32 = strm->total_out_hi32 = 0;
  return BZ_OK;
}

int BZ2_bzCompress(bz_stream* strm, int action) {
  if (strm == nullptr || strm->state == nullptr) return BZ_PARAM_ERROR;
  CState* s = (CState*)strm->state;
  if (s->strm != strm) return BZ_PARAM_ERROR;
  for (;;) {
    switch (s->mode) {
      case kModeIdle:
        return BZ_SEQUENCE_ERROR;
      case kModeRunning:
        if (action == BZ_RUN) {
          bool progress = take_input(s);
          if (s->staged.size() >= s->stage_limit) {
            int rc = run_device(s, false, false);
            if (rc != BZ_OK) return rc;
            s->stage_limit = std::min(2 * s->stage_limit, kStageMax);
          }
          progress |= drain(s);
          return progress ? BZ_RUN_OK : BZ_PARAM_ERROR;
        }
        if (action == BZ_FLUSH || action == BZ_FINISH) {
          s->avail_in_expect = strm->avail_in;
          s->tail_merge = strm->avail_in > 0;
          s->segment_done = false;
          s->mode = action == BZ_FLUSH ? kModeFlushing : kModeFinishing;
          continue;
        }
        return BZ_PARAM_ERROR;
      case kModeFlushing:
      case kModeFinishing: {
        const bool finishing = s->mode == kModeFinishing;
        if (action != (finishing ? BZ_FINISH : BZ_FLUSH)) return BZ_SEQUENCE_ERROR;
        if (s->avail_in_expect != strm->avail_in) return BZ_SEQUENCE_ERROR;
        bool progress = take_input(s);
        s->avail_in_expect = strm->avail_in;
        if (!s->segment_done) {
          int rc = run_device(s, true, finishing);
          if (rc != BZ_OK) return rc;
          s->segment_done = true;
          progress = true;
        }
        progress |= drain(s);
        if (finishing && !progress) return BZ_SEQUENCE_ERROR;
        if (s->out_pos < s->out.size()) return finishing ? BZ_FINISH_OK : BZ_FLUSH_OK;
        if (finishing) {
          s->mode = kModeIdle;
          return BZ_STREAM_END;
        }
        s->mode = kModeRunning;
        return BZ_RUN_OK;
      }
      default:
        return BZ_OK;
    }
  }
}

int BZ2_bzCompressEnd(bz_stream* strm) {
  if (strm == nullptr || strm->state == nullptr) return BZ_PARAM_ERROR;
  CState* s = (CState*)strm->state;
  if (s->strm != strm) return BZ_PARAM_ERROR;
  s->~CState();
  strm->bzfree(strm->opaque, s);
  strm->state = nullptr;
  return BZ_OK;
}

int BZ2_bzBuffToBuffCompress(char* dest, unsigned int* destLen, char* source, unsigned int sourceLen,
                             int blockSize100k, int verbosity, int workFactor) {
  if (dest == nullptr || destLen == nullptr || source == nullptr || blockSize100k < 1 || blockSize100k > 9 ||
      verbosity < 0 || verbosity > 4 || workFactor < 0 || workFactor > 250)
    return BZ_PARAM_ERROR;
  uint64_t len = 0;
  int rc = bzg_compress_host(source, sourceLen, blockSize100k, dest, *destLen, &len);
  if (rc == BZ_OK) *destLen = (unsigned)len;
  return rc;
}

const char* BZ2_bzlibVersion(void) { return "1.0.6x, 16-Aug-2018"; }

}  // extern "C"
