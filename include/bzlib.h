/* bzlib.h -- public ABI of the MI355X bzip2 library (drop-in libbz2.so.1.0).
 *
 * This header declares exactly the interface of the reference's bzlib.h (bzlib.h:1-282 of
 * aeb1787/bzip2 "1.0.6x") and its 24 exports (libbz2.def:4-27); struct layout, constants and
 * prototypes are unchanged so existing callers relink or LD_PRELOAD without source changes.
 * The compression entry points run the hot path on the GPU (see include/bzg.h); the
 * decompression entry points are served by this library's own CPU decoder.
 */
#ifndef _BZLIB_H
#define _BZLIB_H

#ifdef __cplusplus
extern "C" {
#endif

#define BZ_RUN 0
#define BZ_FLUSH 1
#define BZ_FINISH 2

#define BZ_OK 0
#define BZ_RUN_OK 1
#define BZ_FLUSH_OK 2
#define BZ_FINISH_OK 3
#define BZ_STREAM_END 4
#define BZ_SEQUENCE_ERROR (-1)
#define BZ_PARAM_ERROR (-2)
#define BZ_MEM_ERROR (-3)
#define BZ_DATA_ERROR (-4)
#define BZ_DATA_ERROR_MAGIC (-5)
#define BZ_IO_ERROR (-6)
#define BZ_UNEXPECTED_EOF (-7)
#define BZ_OUTBUFF_FULL (-8)
#define BZ_CONFIG_ERROR (-9)

typedef struct {
  char *next_in;
  unsigned int avail_in;
  unsigned int total_in_lo32;
  unsigned int total_in_hi32;

  char *next_out;
  unsigned int avail_out;
  unsigned int total_out_lo32;
  unsigned int total_out_hi32;

  void *state;

  void *(*bzalloc)(void *, int, int);
  void (*bzfree)(void *, void *);
  void *opaque;
} bz_stream;

#ifndef BZ_NO_STDIO
#include <stdio.h>
#endif

#define BZ_API(func) func
#define BZ_EXTERN extern

/* reference bzlib.h:100-114 (core compression) */
BZ_EXTERN int BZ_API(BZ2_bzCompressInit)(bz_stream *strm, int blockSize100k, int verbosity, int workFactor);
BZ_EXTERN int BZ_API(BZ2_bzCompress)(bz_stream *strm, int action);
BZ_EXTERN int BZ_API(BZ2_bzCompressEnd)(bz_stream *strm);

/* reference bzlib.h:116-129 (core decompression) */
BZ_EXTERN int BZ_API(BZ2_bzDecompressInit)(bz_stream *strm, int verbosity, int small);
BZ_EXTERN int BZ_API(BZ2_bzDecompress)(bz_stream *strm);
BZ_EXTERN int BZ_API(BZ2_bzDecompressEnd)(bz_stream *strm);

#ifndef BZ_NO_STDIO
#define BZ_MAX_UNUSED 5000

typedef void BZFILE;

/* reference bzlib.h:139-201 (FILE* layer) */
BZ_EXTERN BZFILE *BZ_API(BZ2_bzReadOpen)(int *bzerror, FILE *f, int verbosity, int small, void *unused, int nUnused);
BZ_EXTERN void BZ_API(BZ2_bzReadClose)(int *bzerror, BZFILE *b);
BZ_EXTERN void BZ_API(BZ2_bzReadGetUnused)(int *bzerror, BZFILE *b, void **unused, int *nUnused);
BZ_EXTERN int BZ_API(BZ2_bzRead)(int *bzerror, BZFILE *b, void *buf, int len);
BZ_EXTERN BZFILE *BZ_API(BZ2_bzWriteOpen)(int *bzerror, FILE *f, int blockSize100k, int verbosity, int workFactor);
BZ_EXTERN void BZ_API(BZ2_bzWrite)(int *bzerror, BZFILE *b, void *buf, int len);
BZ_EXTERN void BZ_API(BZ2_bzWriteClose)(int *bzerror, BZFILE *b, int abandon, unsigned int *nbytes_in,
                                         unsigned int *nbytes_out);
BZ_EXTERN void BZ_API(BZ2_bzWriteClose64)(int *bzerror, BZFILE *b, int abandon, unsigned int *nbytes_in_lo32,
                                           unsigned int *nbytes_in_hi32, unsigned int *nbytes_out_lo32,
                                           unsigned int *nbytes_out_hi32);
#endif

/* reference bzlib.h:204-220 (one-shot buffers) */
BZ_EXTERN int BZ_API(BZ2_bzBuffToBuffCompress)(char *dest, unsigned int *destLen, char *source, unsigned int sourceLen,
                                               int blockSize100k, int verbosity, int workFactor);
BZ_EXTERN int BZ_API(BZ2_bzBuffToBuffDecompress)(char *dest, unsigned int *destLen, char *source,
                                                 unsigned int sourceLen, int small, int verbosity);

/* reference bzlib.h:223-271 (zlib-style helpers) */
BZ_EXTERN const char *BZ_API(BZ2_bzlibVersion)(void);
#ifndef BZ_NO_STDIO
BZ_EXTERN BZFILE *BZ_API(BZ2_bzopen)(const char *path, const char *mode);
BZ_EXTERN BZFILE *BZ_API(BZ2_bzdopen)(int fd, const char *mode);
BZ_EXTERN int BZ_API(BZ2_bzread)(BZFILE *b, void *buf, int len);
BZ_EXTERN int BZ_API(BZ2_bzwrite)(BZFILE *b, void *buf, int len);
BZ_EXTERN int BZ_API(BZ2_bzflush)(BZFILE *b);
BZ_EXTERN void BZ_API(BZ2_bzclose)(BZFILE *b);
BZ_EXTERN const char *BZ_API(BZ2_bzerror)(BZFILE *b, int *errnum);
#endif

#ifdef __cplusplus
}
#endif

#endif
