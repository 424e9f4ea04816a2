// bzlib_api.cpp -- the 24 exports of libbz2.def (reference libbz2.def:4-27) over the GPU engine.
//
// Compression keeps the reference's streaming contract (bzlib.c:144-474): BZ_RUN returns
// BZ_RUN_OK iff progress was made, BZ_FLUSH / BZ_FINISH move the stream into FLUSHING /
// FINISHING and must be repeated with an unchanged avail_in until BZ_RUN_OK / BZ_STREAM_END.
// Input is staged on the host and compressed by the device in batches; output may lag input
// (the concatenated bytes are what the reference emits for the same call pattern):
//   * RUN-mode bytes are staged; once kStageMax bytes are staged the complete blocks among
//     them are compressed (RUN semantics: a full block is cut, bzlib.c:383-386);
//   * FLUSH / FINISH compress everything staged as the end of a segment; the final length-1
//     run chunk joins a full block only when bytes arrived with the FLUSH/FINISH call
//     (bzlib.c:276-308).
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
          if (s->staged.size() >= kStageMax) {
            int rc = run_device(s, false, false);
            if (rc != BZ_OK) return rc;
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

// ------------------------------------------------------------------ FILE* layer
// Restates bzlib.c:943-1301 over the stream functions above and the decoder.
struct BzFile {
  FILE* handle;
  char buf[BZ_MAX_UNUSED];
  int bufN;
  bool writing;
  bz_stream strm;
  int lastErr;
  bool initialisedOk;
};

#define BZ_SETERR(eee)                    \
  do {                                    \
    if (bzerror != nullptr) *bzerror = eee; \
    if (bzf != nullptr) bzf->lastErr = eee; \
  } while (0)

static bool my_feof(FILE* f) {
  int c = fgetc(f);
  if (c == EOF) return true;
  ungetc(c, f);
  return false;
}

BZFILE* BZ2_bzWriteOpen(int* bzerror, FILE* f, int blockSize100k, int verbosity, int workFactor) {
  BzFile* bzf = nullptr;
  BZ_SETERR(BZ_OK);
  if (f == nullptr || blockSize100k < 1 || blockSize100k > 9 || workFactor < 0 || workFactor > 250 ||
      verbosity < 0 || verbosity > 4) {
    BZ_SETERR(BZ_PARAM_ERROR);
    return nullptr;
  }
  if (ferror(f)) {
    BZ_SETERR(BZ_IO_ERROR);
    return nullptr;
  }
  bzf = (BzFile*)std::malloc(sizeof(BzFile));
  if (bzf == nullptr) {
    BZ_SETERR(BZ_MEM_ERROR);
    return nullptr;
  }
  BZ_SETERR(BZ_OK);
  bzf->initialisedOk = false;
  bzf->bufN = 0;
  bzf->handle = f;
  bzf->writing = true;
  bzf->strm.bzalloc = nullptr;
  bzf->strm.bzfree = nullptr;
  bzf->strm.opaque = nullptr;
  if (workFactor == 0) workFactor = 30;
  int ret = BZ2_bzCompressInit(&bzf->strm, blockSize100k, verbosity, workFactor);
  if (ret != BZ_OK) {
    BZ_SETERR(ret);
    std::free(bzf);
    return nullptr;
  }
  bzf->strm.avail_in = 0;
  bzf->initialisedOk = true;
  return bzf;
}

void BZ2_bzWrite(int* bzerror, BZFILE* b, void* buf, int len) {
  BzFile* bzf = (BzFile*)b;
  BZ_SETERR(BZ_OK);
  if (bzf == nullptr || buf == nullptr || len < 0) {
    BZ_SETERR(BZ_PARAM_ERROR);
    return;
  }
  if (!bzf->writing) {
    BZ_SETERR(BZ_SEQUENCE_ERROR);
    return;
  }
  if (ferror(bzf->handle)) {
    BZ_SETERR(BZ_IO_ERROR);
    return;
  }
  if (len == 0) {
    BZ_SETERR(BZ_OK);
    return;
  }
  bzf->strm.avail_in = (unsigned)len;
  bzf->strm.next_in = (char*)buf;
  for (;;) {
    bzf->strm.avail_out = BZ_MAX_UNUSED;
    bzf->strm.next_out = bzf->buf;
    int ret = BZ2_bzCompress(&bzf->strm, BZ_RUN);
    if (ret != BZ_RUN_OK) {
      BZ_SETERR(ret);
      return;
    }
    if (bzf->strm.avail_out < BZ_MAX_UNUSED) {
      size_t n = BZ_MAX_UNUSED - bzf->strm.avail_out;
      size_t n2 = fwrite(bzf->buf, 1, n, bzf->handle);
      if (n != n2 || ferror(bzf->handle)) {
        BZ_SETERR(BZ_IO_ERROR);
        return;
      }
    }
    if (bzf->strm.avail_in == 0) {
      BZ_SETERR(BZ_OK);
      return;
    }
  }
}

void BZ2_bzWriteClose64(int* bzerror, BZFILE* b, int abandon, unsigned int* nbytes_in_lo32,
                        unsigned int* nbytes_in_hi32, unsigned int* nbytes_out_lo32, unsigned int* nbytes_out_hi32) {
  BzFile* bzf = (BzFile*)b;
  if (bzf == nullptr) {
    BZ_SETERR(BZ_OK);
    return;
  }
  if (!bzf->writing) {
    BZ_SETERR(BZ_SEQUENCE_ERROR);
    return;
  }
  if (ferror(bzf->handle)) {
    BZ_SETERR(BZ_IO_ERROR);
    return;
  }
  if (nbytes_in_lo32) *nbytes_in_lo32 = 0;
  if (nbytes_in_hi32) *nbytes_in_hi32 = 0;
  if (nbytes_out_lo32) *nbytes_out_lo32 = 0;
  if (nbytes_out_hi32) *nbytes_out_hi32 = 0;
  if (!abandon && bzf->lastErr == BZ_OK) {
    for (;;) {
      bzf->strm.avail_out = BZ_MAX_UNUSED;
      bzf->strm.next_out = bzf->buf;
      int ret = BZ2_bzCompress(&bzf->strm, BZ_FINISH);
      if (ret != BZ_FINISH_OK && ret != BZ_STREAM_END) {
        BZ_SETERR(ret);
        return;
      }
      if (bzf->strm.avail_out < BZ_MAX_UNUSED) {
        size_t n = BZ_MAX_UNUSED - bzf->strm.avail_out;
        size_t n2 = fwrite(bzf->buf, 1, n, bzf->handle);
        if (n != n2 || ferror(bzf->handle)) {
          BZ_SETERR(BZ_IO_ERROR);
          return;
        }
      }
      if (ret == BZ_STREAM_END) break;
    }
  }
  if (!abandon && !ferror(bzf->handle)) {
    fflush(bzf->handle);
    if (ferror(bzf->handle)) {
      BZ_SETERR(BZ_IO_ERROR);
      return;
    }
  }
  if (nbytes_in_lo32) *nbytes_in_lo32 = bzf->strm.total_in_lo32;
  if (nbytes_in_hi32) *nbytes_in_hi32 = bzf->strm.total_in_hi32;
  if (nbytes_out_lo32) *nbytes_out_lo32 = bzf->strm.total_out_lo32;
  if (nbytes_out_hi32) *nbytes_out_hi32 = bzf->strm.total_out_hi32;
  BZ_SETERR(BZ_OK);
  BZ2_bzCompressEnd(&bzf->strm);
  std::free(bzf);
}

void BZ2_bzWriteClose(int* bzerror, BZFILE* b, int abandon, unsigned int* nbytes_in, unsigned int* nbytes_out) {
  BZ2_bzWriteClose64(bzerror, b, abandon, nbytes_in, nullptr, nbytes_out, nullptr);
}

BZFILE* BZ2_bzReadOpen(int* bzerror, FILE* f, int verbosity, int small, void* unused, int nUnused) {
  BzFile* bzf = nullptr;
  BZ_SETERR(BZ_OK);
  if (f == nullptr || (small != 0 && small != 1) || verbosity < 0 || verbosity > 4 ||
      (unused == nullptr && nUnused != 0) || (unused != nullptr && (nUnused < 0 || nUnused > BZ_MAX_UNUSED))) {
    BZ_SETERR(BZ_PARAM_ERROR);
    return nullptr;
  }
  if (ferror(f)) {
    BZ_SETERR(BZ_IO_ERROR);
    return nullptr;
  }
  bzf = (BzFile*)std::malloc(sizeof(BzFile));
  if (bzf == nullptr) {
    BZ_SETERR(BZ_MEM_ERROR);
    return nullptr;
  }
  BZ_SETERR(BZ_OK);
  bzf->initialisedOk = false;
  bzf->handle = f;
  bzf->bufN = 0;
  bzf->writing = false;
  bzf->strm.bzalloc = nullptr;
  bzf->strm.bzfree = nullptr;
  bzf->strm.opaque = nullptr;
  while (nUnused > 0) {
    bzf->buf[bzf->bufN++] = *(char*)unused;
    unused = (char*)unused + 1;
    nUnused--;
  }
  int ret = BZ2_bzDecompressInit(&bzf->strm, verbosity, small);
  if (ret != BZ_OK) {
    BZ_SETERR(ret);
    std::free(bzf);
    return nullptr;
  }
  bzf->strm.avail_in = (unsigned)bzf->bufN;
  bzf->strm.next_in = bzf->buf;
  bzf->initialisedOk = true;
  return bzf;
}

void BZ2_bzReadClose(int* bzerror, BZFILE* b) {
  BzFile* bzf = (BzFile*)b;
  BZ_SETERR(BZ_OK);
  if (bzf == nullptr) {
    BZ_SETERR(BZ_OK);
    return;
  }
  if (bzf->writing) {
    BZ_SETERR(BZ_SEQUENCE_ERROR);
    return;
  }
  if (bzf->initialisedOk) (void)BZ2_bzDecompressEnd(&bzf->strm);
  std::free(bzf);
}

int BZ2_bzRead(int* bzerror, BZFILE* b, void* buf, int len) {
  BzFile* bzf = (BzFile*)b;
  BZ_SETERR(BZ_OK);
  if (bzf == nullptr || buf == nullptr || len < 0) {
    BZ_SETERR(BZ_PARAM_ERROR);
    return 0;
  }
  if (bzf->writing) {
    BZ_SETERR(BZ_SEQUENCE_ERROR);
    return 0;
  }
  if (len == 0) {
    BZ_SETERR(BZ_OK);
    return 0;
  }
  bzf->strm.avail_out = (unsigned)len;
  bzf->strm.next_out = (char*)buf;
  for (;;) {
    if (ferror(bzf->handle)) {
      BZ_SETERR(BZ_IO_ERROR);
      return 0;
    }
    if (bzf->strm.avail_in == 0 && !my_feof(bzf->handle)) {
      size_t n = fread(bzf->buf, 1, BZ_MAX_UNUSED, bzf->handle);
      if (ferror(bzf->handle)) {
        BZ_SETERR(BZ_IO_ERROR);
        return 0;
      }
      bzf->bufN = (int)n;
      bzf->strm.avail_in = (unsigned)bzf->bufN;
      bzf->strm.next_in = bzf->buf;
    }
    int ret = BZ2_bzDecompress(&bzf->strm);
    if (ret != BZ_OK && ret != BZ_STREAM_END) {
      BZ_SETERR(ret);
      return 0;
    }
    if (ret == BZ_OK && my_feof(bzf->handle) && bzf->strm.avail_in == 0 && bzf->strm.avail_out > 0) {
      BZ_SETERR(BZ_UNEXPECTED_EOF);
      return 0;
    }
    if (ret == BZ_STREAM_END) {
      BZ_SETERR(BZ_STREAM_END);
      return len - (int)bzf->strm.avail_out;
    }
    if (bzf->strm.avail_out == 0) {
      BZ_SETERR(BZ_OK);
      return len;
    }
  }
}

void BZ2_bzReadGetUnused(int* bzerror, BZFILE* b, void** unused, int* nUnused) {
  BzFile* bzf = (BzFile*)b;
  if (bzf == nullptr) {
    BZ_SETERR(BZ_PARAM_ERROR);
    return;
  }
  if (bzf->lastErr != BZ_STREAM_END) {
    BZ_SETERR(BZ_SEQUENCE_ERROR);
    return;
  }
  if (unused == nullptr || nUnused == nullptr) {
    BZ_SETERR(BZ_PARAM_ERROR);
    return;
  }
  BZ_SETERR(BZ_OK);
  *nUnused = (int)bzf->strm.avail_in;
  *unused = bzf->strm.next_in;
}

int BZ2_bzBuffToBuffDecompress(char* dest, unsigned int* destLen, char* source, unsigned int sourceLen, int small,
                               int verbosity) {
  if (dest == nullptr || destLen == nullptr || source == nullptr || (small != 0 && small != 1) || verbosity < 0 ||
      verbosity > 4)
    return BZ_PARAM_ERROR;
  bz_stream strm;
  strm.bzalloc = nullptr;
  strm.bzfree = nullptr;
  strm.opaque = nullptr;
  int ret = BZ2_bzDecompressInit(&strm, verbosity, small);
  if (ret != BZ_OK) return ret;
  strm.next_in = source;
  strm.next_out = dest;
  strm.avail_in = sourceLen;
  strm.avail_out = *destLen;
  ret = BZ2_bzDecompress(&strm);
  if (ret == BZ_OK) {
    const bool eof = strm.avail_out > 0;
    BZ2_bzDecompressEnd(&strm);
    return eof ? BZ_UNEXPECTED_EOF : BZ_OUTBUFF_FULL;
  }
  if (ret != BZ_STREAM_END) {
    BZ2_bzDecompressEnd(&strm);
    return ret;
  }
  *destLen -= strm.avail_out;
  BZ2_bzDecompressEnd(&strm);
  return BZ_OK;
}

// zlib-style helpers (bzlib.c:1445-1628)
static BZFILE* bzopen_or_bzdopen(const char* path, int fd, const char* mode, int open_mode) {
  int bzerr;
  char unused[BZ_MAX_UNUSED];
  int blockSize100k = 9;
  int writing = 0;
  char mode2[10] = "";
  FILE* fp = nullptr;
  BZFILE* bzfp = nullptr;
  int verbosity = 0, workFactor = 30, smallMode = 0, nUnused = 0;
  if (mode == nullptr) return nullptr;
  while (*mode) {
    switch (*mode) {
      case 'r': writing = 0; break;
      case 'w': writing = 1; break;
      case 's': smallMode = 1; break;
      default:
        if (*mode >= '0' && *mode <= '9') blockSize100k = *mode - '0';
    }
    mode++;
  }
  std::strcat(mode2, writing ? "w" : "r");
  std::strcat(mode2, "b");
  if (open_mode == 0) {
    if (path == nullptr || std::strcmp(path, "") == 0) fp = writing ? stdout : stdin;
    else fp = fopen(path, mode2);
  } else {
    fp = fdopen(fd, mode2);
  }
  if (fp == nullptr) return nullptr;
  if (writing) {
    if (blockSize100k < 1) blockSize100k = 1;
    if (blockSize100k > 9) blockSize100k = 9;
    bzfp = BZ2_bzWriteOpen(&bzerr, fp, blockSize100k, verbosity, workFactor);
  } else {
    bzfp = BZ2_bzReadOpen(&bzerr, fp, verbosity, smallMode, unused, nUnused);
  }
  if (bzfp == nullptr) {
    if (fp != stdin && fp != stdout) fclose(fp);
    return nullptr;
  }
  return bzfp;
}

BZFILE* BZ2_bzopen(const char* path, const char* mode) { return bzopen_or_bzdopen(path, -1, mode, 0); }
BZFILE* BZ2_bzdopen(int fd, const char* mode) { return bzopen_or_bzdopen(nullptr, fd, mode, 1); }

int BZ2_bzread(BZFILE* b, void* buf, int len) {
  int bzerr;
  if (((BzFile*)b)->lastErr == BZ_STREAM_END) return 0;
  int nread = BZ2_bzRead(&bzerr, b, buf, len);
  return (bzerr == BZ_OK || bzerr == BZ_STREAM_END) ? nread : -1;
}

int BZ2_bzwrite(BZFILE* b, void* buf, int len) {
  int bzerr;
  BZ2_bzWrite(&bzerr, b, buf, len);
  return bzerr == BZ_OK ? len : -1;
}

int BZ2_bzflush(BZFILE*) { return 0; }

void BZ2_bzclose(BZFILE* b) {
  int bzerr;
  if (b == nullptr) return;
  FILE* fp = ((BzFile*)b)->handle;
  if (((BzFile*)b)->writing) {
    BZ2_bzWriteClose(&bzerr, b, 0, nullptr, nullptr);
    if (bzerr != BZ_OK) BZ2_bzWriteClose(nullptr, b, 1, nullptr, nullptr);
  } else {
    BZ2_bzReadClose(&bzerr, b);
  }
  if (fp != stdin && fp != stdout) fclose(fp);
}

static const char* kErrStr[] = {"OK",         "SEQUENCE_ERROR", "PARAM_ERROR",    "MEM_ERROR",
                                "DATA_ERROR", "DATA_ERROR_MAGIC", "IO_ERROR",     "UNEXPECTED_EOF",
                                "OUTBUFF_FULL", "CONFIG_ERROR", "???",            "???",
                                "???",        "???",            "???",            "???"};

const char* BZ2_bzerror(BZFILE* b, int* errnum) {
  int err = ((BzFile*)b)->lastErr;
  if (err > 0) err = 0;
  *errnum = err;
  return kErrStr[err * -1];
}

}  // extern "C"
