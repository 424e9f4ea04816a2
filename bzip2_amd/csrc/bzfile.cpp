// bzfile.cpp -- the stdio and zlib-style exports of libbz2.def over the stream functions
// (BZ2_bzWriteOpen .. BZ2_bzerror, BZ2_bzBuffToBuffDecompress).
//
// Interface and error behaviour follow the reference's bzlib.h:140-282 / bzlib.c:943-1628:
//   * every entry point that takes `int* bzerror` stores its outcome there (when non-null) and
//     in the handle (read back by BZ2_bzerror and by BZ2_bzRead/ReadGetUnused);
//   * argument errors are BZ_PARAM_ERROR, using a handle in the wrong direction is
//     BZ_SEQUENCE_ERROR, a stdio failure is BZ_IO_ERROR, a compressed file that ends early
//     is BZ_UNEXPECTED_EOF;
//   * close on a null handle is a no-op with BZ_OK.
// Compression goes through BZ2_bzCompress (the GPU engine), stream decompression through the
// library's CPU decoder (BZ2_bzBuffToBuffDecompress uses the GPU decoder); both are driven through a BZ_MAX_UNUSED-byte staging buffer as the
// reference does, so the bytes written to the FILE are exactly those of the stream calls.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "../../include/bzg.h"
#include "../../include/bzlib.h"

namespace {

enum class Dir { kWrite, kRead };

class BzHandle {
 public:
  BzHandle(FILE* f, Dir d) : file_(f), dir_(d) {
    std::memset(&strm_, 0, sizeof(strm_));
  }

  FILE* file() const { return file_; }
  bool writing() const { return dir_ == Dir::kWrite; }
  int last_error() const { return last_; }
  void set_error(int e) { last_ = e; }
  bz_stream& strm() { return strm_; }

  // ---- writing side
  int open_writer(int level, int verbosity, int work) {
    const int rc = BZ2_bzCompressInit(&strm_, level, verbosity, work == 0 ? 30 : work);
    live_ = rc == BZ_OK;
    return rc;
  }

  // Pushes len bytes through BZ_RUN; whatever the stream hands back goes to the file.
  int write(const char* buf, int len) {
    strm_.next_in = const_cast<char*>(buf);
    strm_.avail_in = (unsigned)len;
    while (strm_.avail_in > 0) {
      const int rc = pump(BZ_RUN);
      if (rc != BZ_RUN_OK) return rc;
      if (!flush_staging()) return BZ_IO_ERROR;
    }
    return BZ_OK;
  }

  // BZ_FINISH until the stream ends, every piece written out.
  int finish() {
    for (;;) {
      const int rc = pump(BZ_FINISH);
      if (rc != BZ_FINISH_OK && rc != BZ_STREAM_END) return rc;
      if (!flush_staging()) return BZ_IO_ERROR;
      if (rc == BZ_STREAM_END) return BZ_OK;
    }
  }

  void end_writer() {
    if (live_) BZ2_bzCompressEnd(&strm_);
    live_ = false;
  }

  // ---- reading side
  int open_reader(int verbosity, int small, const char* unused, int n_unused) {
    if (n_unused > 0) std::memcpy(stage_, unused, (size_t)n_unused);
    const int rc = BZ2_bzDecompressInit(&strm_, verbosity, small);
    if (rc != BZ_OK) return rc;
    live_ = true;
    strm_.next_in = stage_;
    strm_.avail_in = (unsigned)n_unused;
    return BZ_OK;
  }

  // Decodes up to len bytes into buf; *got = bytes produced.  Returns BZ_OK, BZ_STREAM_END or
  // an error code.
  int read(char* buf, int len, int* got) {
    *got = 0;
    strm_.next_out = buf;
    strm_.avail_out = (unsigned)len;
    for (;;) {
      if (std::ferror(file_)) return BZ_IO_ERROR;
      if (strm_.avail_in == 0 && !at_eof()) {
        const size_t n = std::fread(stage_, 1, BZ_MAX_UNUSED, file_);
        if (std::ferror(file_)) return BZ_IO_ERROR;
        strm_.next_in = stage_;
        strm_.avail_in = (unsigned)n;
      }
      const int rc = BZ2_bzDecompress(&strm_);
      *got = len - (int)strm_.avail_out;
      if (rc == BZ_STREAM_END) return BZ_STREAM_END;
      if (rc != BZ_OK) {
        *got = 0;
        return rc;
      }
      if (strm_.avail_out == 0) return BZ_OK;
      if (strm_.avail_in == 0 && at_eof()) {
        *got = 0;
        return BZ_UNEXPECTED_EOF;
      }
    }
  }

  void end_reader() {
    if (live_) BZ2_bzDecompressEnd(&strm_);
    live_ = false;
  }

 private:
  int pump(int action) {
    strm_.next_out = stage_;
    strm_.avail_out = BZ_MAX_UNUSED;
    return BZ2_bzCompress(&strm_, action);
  }

  bool flush_staging() {
    const size_t n = BZ_MAX_UNUSED - strm_.avail_out;
    if (n == 0) return !std::ferror(file_);
    return std::fwrite(stage_, 1, n, file_) == n && !std::ferror(file_);
  }

  bool at_eof() {
    const int c = std::fgetc(file_);
    if (c == EOF) return true;
    std::ungetc(c, file_);
    return false;
  }

  FILE* file_;
  Dir dir_;
  bz_stream strm_;
  bool live_ = false;
  int last_ = BZ_OK;
  char stage_[BZ_MAX_UNUSED];
};

// Outcome of one call: into *bzerror (if given) and into the handle (if any).
struct Outcome {
  int* out;
  BzHandle* h;
  void operator()(int code) const {
    if (out) *out = code;
    if (h) h->set_error(code);
  }
};

BzHandle* as_handle(BZFILE* b) { return static_cast<BzHandle*>(b); }

const char* error_name(int code) {
  switch (code) {
    case BZ_OK: return "OK";
    case BZ_SEQUENCE_ERROR: return "SEQUENCE_ERROR";
    case BZ_PARAM_ERROR: return "PARAM_ERROR";
    case BZ_MEM_ERROR: return "MEM_ERROR";
    case BZ_DATA_ERROR: return "DATA_ERROR";
    case BZ_DATA_ERROR_MAGIC: return "DATA_ERROR_MAGIC";
    case BZ_IO_ERROR: return "IO_ERROR";
    case BZ_UNEXPECTED_EOF: return "UNEXPECTED_EOF";
    case BZ_OUTBUFF_FULL: return "OUTBUFF_FULL";
    case BZ_CONFIG_ERROR: return "CONFIG_ERROR";
    default: return "???";
  }
}

// Mode string of BZ2_bzopen: 'r' / 'w' pick the direction (last one wins), 's' the small
// decoder, a digit the block size; anything else is ignored.
struct OpenMode {
  bool write = false;
  bool small = false;
  int level = 9;
  explicit OpenMode(const char* m) {
    for (; *m; ++m) {
      if (*m == 'r') write = false;
      else if (*m == 'w') write = true;
      else if (*m == 's') small = true;
      else if (*m >= '0' && *m <= '9') level = *m - '0';
    }
    if (level < 1) level = 1;
  }
};

BZFILE* open_common(FILE* fp, const OpenMode& om) {
  int err = BZ_OK;
  if (om.write) return BZ2_bzWriteOpen(&err, fp, om.level, 0, 30);
  return BZ2_bzReadOpen(&err, fp, 0, om.small ? 1 : 0, nullptr, 0);
}

BZFILE* open_stdio(FILE* fp, const OpenMode& om) {
  if (!fp) return nullptr;
  BZFILE* b = open_common(fp, om);
  if (!b && fp != stdin && fp != stdout) std::fclose(fp);
  return b;
}

}  // namespace

extern "C" {

BZFILE* BZ2_bzWriteOpen(int* bzerror, FILE* f, int blockSize100k, int verbosity, int workFactor) {
  Outcome done{bzerror, nullptr};
  if (!f || blockSize100k < 1 || blockSize100k > 9 || workFactor < 0 || workFactor > 250 || verbosity < 0 ||
      verbosity > 4) {
    done(BZ_PARAM_ERROR);
    return nullptr;
  }
  if (std::ferror(f)) {
    done(BZ_IO_ERROR);
    return nullptr;
  }
  BzHandle* h = new (std::nothrow) BzHandle(f, Dir::kWrite);
  if (!h) {
    done(BZ_MEM_ERROR);
    return nullptr;
  }
  const int rc = h->open_writer(blockSize100k, verbosity, workFactor);
  if (rc != BZ_OK) {
    delete h;
    done(rc);
    return nullptr;
  }
  done(BZ_OK);
  return h;
}

void BZ2_bzWrite(int* bzerror, BZFILE* b, void* buf, int len) {
  BzHandle* h = as_handle(b);
  Outcome done{bzerror, h};
  if (!h || !buf || len < 0) return done(BZ_PARAM_ERROR);
  if (!h->writing()) return done(BZ_SEQUENCE_ERROR);
  if (std::ferror(h->file())) return done(BZ_IO_ERROR);
  if (len == 0) return done(BZ_OK);
  done(h->write(static_cast<const char*>(buf), len));
}

void BZ2_bzWriteClose64(int* bzerror, BZFILE* b, int abandon, unsigned int* nbytes_in_lo32,
                        unsigned int* nbytes_in_hi32, unsigned int* nbytes_out_lo32, unsigned int* nbytes_out_hi32) {
  BzHandle* h = as_handle(b);
  Outcome done{bzerror, h};
  if (!h) return done(BZ_OK);
  if (!h->writing()) return done(BZ_SEQUENCE_ERROR);
  if (std::ferror(h->file())) return done(BZ_IO_ERROR);
  unsigned int* counters[4] = {nbytes_in_lo32, nbytes_in_hi32, nbytes_out_lo32, nbytes_out_hi32};
  for (unsigned int* c : counters)
    if (c) *c = 0;
  if (!abandon && h->last_error() == BZ_OK) {
    const int rc = h->finish();
    if (rc != BZ_OK) return done(rc);
  }
  if (!abandon && !std::ferror(h->file())) {
    std::fflush(h->file());
    if (std::ferror(h->file())) return done(BZ_IO_ERROR);
  }
  const bz_stream& z = h->strm();
  const unsigned int vals[4] = {z.total_in_lo32, z.total_in_hi32, z.total_out_lo32, z.total_out_hi32};
  for (int i = 0; i < 4; i++)
    if (counters[i]) *counters[i] = vals[i];
  if (bzerror) *bzerror = BZ_OK;
  h->end_writer();
  delete h;
}

void BZ2_bzWriteClose(int* bzerror, BZFILE* b, int abandon, unsigned int* nbytes_in, unsigned int* nbytes_out) {
  BZ2_bzWriteClose64(bzerror, b, abandon, nbytes_in, nullptr, nbytes_out, nullptr);
}

BZFILE* BZ2_bzReadOpen(int* bzerror, FILE* f, int verbosity, int small, void* unused, int nUnused) {
  Outcome done{bzerror, nullptr};
  const bool bad_unused = unused ? (nUnused < 0 || nUnused > BZ_MAX_UNUSED) : nUnused != 0;
  if (!f || (small != 0 && small != 1) || verbosity < 0 || verbosity > 4 || bad_unused) {
    done(BZ_PARAM_ERROR);
    return nullptr;
  }
  if (std::ferror(f)) {
    done(BZ_IO_ERROR);
    return nullptr;
  }
  BzHandle* h = new (std::nothrow) BzHandle(f, Dir::kRead);
  if (!h) {
    done(BZ_MEM_ERROR);
    return nullptr;
  }
  const int rc = h->open_reader(verbosity, small, static_cast<const char*>(unused), unused ? nUnused : 0);
  if (rc != BZ_OK) {
    delete h;
    done(rc);
    return nullptr;
  }
  done(BZ_OK);
  return h;
}

void BZ2_bzReadClose(int* bzerror, BZFILE* b) {
  BzHandle* h = as_handle(b);
  Outcome done{bzerror, h};
  if (!h) return done(BZ_OK);
  if (h->writing()) return done(BZ_SEQUENCE_ERROR);
  if (bzerror) *bzerror = BZ_OK;
  h->end_reader();
  delete h;
}

int BZ2_bzRead(int* bzerror, BZFILE* b, void* buf, int len) {
  BzHandle* h = as_handle(b);
  Outcome done{bzerror, h};
  if (!h || !buf || len < 0) {
    done(BZ_PARAM_ERROR);
    return 0;
  }
  if (h->writing()) {
    done(BZ_SEQUENCE_ERROR);
    return 0;
  }
  if (len == 0) {
    done(BZ_OK);
    return 0;
  }
  int got = 0;
  done(h->read(static_cast<char*>(buf), len, &got));
  return got;
}

void BZ2_bzReadGetUnused(int* bzerror, BZFILE* b, void** unused, int* nUnused) {
  BzHandle* h = as_handle(b);
  Outcome done{bzerror, h};
  if (!h) return done(BZ_PARAM_ERROR);
  if (h->last_error() != BZ_STREAM_END) return done(BZ_SEQUENCE_ERROR);
  if (!unused || !nUnused) return done(BZ_PARAM_ERROR);
  done(BZ_OK);
  *nUnused = (int)h->strm().avail_in;
  *unused = h->strm().next_in;
}

int BZ2_bzBuffToBuffDecompress(char* dest, unsigned int* destLen, char* source, unsigned int sourceLen, int small,
                               int verbosity) {
  if (!dest || !destLen || !source || (small != 0 && small != 1) || verbosity < 0 || verbosity > 4)
    return BZ_PARAM_ERROR;
  // Whole in-memory streams decode on the GPU (decomp.hip, all blocks in parallel); the
  // small-memory mode (small = 1) and GPU-less hosts use the library's bit-serial decoder.
  static const bool force_cpu = std::getenv("BZG_CPU_DECODE") != nullptr;
  if (!small && !force_cpu && bzg_device_ok()) {
    uint64_t got = 0;
    const int g = bzg_decompress_host(source, sourceLen, dest, *destLen, &got);
    if (g == BZ_OK) *destLen = (unsigned)got;
    // a device that cannot hold the decode workspace (or fails) leaves the stream to the
    // CPU decoder below, which needs only the caller's buffers
    if (g != BZ_MEM_ERROR && g != BZ_CONFIG_ERROR) return g;
  }
  bz_stream z;
  std::memset(&z, 0, sizeof(z));
  int rc = BZ2_bzDecompressInit(&z, verbosity, small);
  if (rc != BZ_OK) return rc;
  z.next_in = source;
  z.avail_in = sourceLen;
  z.next_out = dest;
  z.avail_out = *destLen;
  rc = BZ2_bzDecompress(&z);
  const unsigned left = z.avail_out;
  BZ2_bzDecompressEnd(&z);
  switch (rc) {
    case BZ_STREAM_END:
      *destLen -= left;
      return BZ_OK;
    case BZ_OK:  // the decoder wants more: either the input ended early or the output is full
      return left > 0 ? BZ_UNEXPECTED_EOF : BZ_OUTBUFF_FULL;
    default:
      return rc;
  }
}

BZFILE* BZ2_bzopen(const char* path, const char* mode) {
  if (!mode) return nullptr;
  const OpenMode om(mode);
  FILE* fp = (!path || !*path) ? (om.write ? stdout : stdin) : std::fopen(path, om.write ? "wb" : "rb");
  return open_stdio(fp, om);
}

BZFILE* BZ2_bzdopen(int fd, const char* mode) {
  if (!mode) return nullptr;
  const OpenMode om(mode);
  return open_stdio(fdopen(fd, om.write ? "wb" : "rb"), om);
}

int BZ2_bzread(BZFILE* b, void* buf, int len) {
  if (as_handle(b)->last_error() == BZ_STREAM_END) return 0;
  int err = BZ_OK;
  const int n = BZ2_bzRead(&err, b, buf, len);
  return (err == BZ_OK || err == BZ_STREAM_END) ? n : -1;
}

int BZ2_bzwrite(BZFILE* b, void* buf, int len) {
  int err = BZ_OK;
  BZ2_bzWrite(&err, b, buf, len);
  return err == BZ_OK ? len : -1;
}

int BZ2_bzflush(BZFILE*) { return 0; }  // the reference's bzflush does nothing either

void BZ2_bzclose(BZFILE* b) {
  BzHandle* h = as_handle(b);
  if (!h) return;
  FILE* fp = h->file();
  int err = BZ_OK;
  if (h->writing()) {
    BZ2_bzWriteClose(&err, b, 0, nullptr, nullptr);
    if (err != BZ_OK) BZ2_bzWriteClose(nullptr, b, 1, nullptr, nullptr);
  } else {
    BZ2_bzReadClose(&err, b);
  }
  if (fp != stdin && fp != stdout) std::fclose(fp);
}

const char* BZ2_bzerror(BZFILE* b, int* errnum) {
  int e = as_handle(b)->last_error();
  if (e > 0) e = 0;
  *errnum = e;
  return error_name(e);
}

}  // extern "C"
