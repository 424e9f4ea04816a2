/* bz_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded restatement of the reference's compression path
 * (aeb1787/bzip2 "1.0.6x"), written from the reference's behaviour, used as the per-stage
 * checker for the HIP kernels.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product library never links or calls it.
 *
 * Parity pinning: every entry point is checked in tests/test_oracle.py against the
 * reference's golden vectors (sample{1,2,3}.bz2, reference Makefile:56-70) and against the
 * reference library itself built from /root/reference by oracle/Makefile (oracle/_ref).
 *
 * One stage is NOT restated: the tie order of identical rotations in exactly periodic
 * blocks is an emergent property of the reference's
 * divsufsort internals; the oracle delegates that single value (origPtr of a periodic
 * block) to a resolver callback, which the tests bind to the reference build.
 */
#ifndef BZ_ORACLE_H
#define BZ_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* CRC-32, MSB-first, polynomial 0x04C11DB7 (bzlib_private.h:187-202, crctable.c). */
uint32_t orc_crc_table(int i);
uint32_t orc_crc_update(uint32_t crc, const uint8_t *p, uint64_t n);

/* RLE1 + block segmentation (bzlib.c:211-315, handle_compress 361-396).
 * tail_merge = 1 reproduces FINISH-with-input (BZ2_bzBuffToBuffCompress): a final length-1
 * run chunk joins a block that is already full; tail_merge = 0 reproduces RUN...then
 * FINISH with avail_in == 0.  Writes concatenated block bytes to blocks (capacity
 * blocks_cap), block byte offsets to blk_off[0..nb], block CRCs to blk_crc[0..nb).
 * Returns the number of blocks, or -1 on overflow. */
int64_t orc_rle1(const uint8_t *in, uint64_t n, int level, int tail_merge,
                 uint8_t *blocks, uint64_t blocks_cap,
                 uint64_t *blk_off, uint32_t *blk_crc, int64_t max_blocks);

/* Resolver for the origPtr of an exactly periodic block (see header comment). */
typedef int (*orc_resolver_fn)(const uint8_t *blk, int n, uint8_t *scratch);
void orc_set_resolver(orc_resolver_fn fn);

/* Cyclic BWT of one block (blocksort.c:1534-1545 semantics): bwt[i] = last column of the
 * i-th smallest rotation; returns origPtr (rank of rotation 0), or -1 if the block is
 * periodic and no resolver is set.  *period_out gets the primitive period p (p == n when
 * aperiodic). */
int orc_bwt(const uint8_t *blk, int n, uint8_t *bwt, int *period_out);

/* MTF + RUNA/RUNB coding (compress.c:93-229).  mtfv needs n+1 entries; freq 258 entries.
 * Returns nMTF; *n_in_use gets nInUse. */
int orc_mtf(const uint8_t *bwt, int n, uint16_t *mtfv, int32_t *freq, int *n_in_use);

/* Heap Huffman code lengths with the reference tie order (huffman.c:63-148). */
void orc_code_lengths(int32_t *len, const int32_t *freq, int alpha, int max_len);

/* Table optimisation + emission of one block's payload (compress.c:250-818).  Bits are
 * appended MSB-first to the writer; sel_out (if not NULL, >= 18002 entries) receives the
 * selectors and *n_sel their count. */
typedef struct {
  uint8_t *buf;
  uint64_t cap;
  uint64_t nbits;
} orc_bits;
void orc_put(orc_bits *w, int nbits, uint32_t v);
int orc_send_mtf(orc_bits *w, const uint16_t *mtfv, int n_mtf, const int32_t *freq,
                 int n_in_use, const uint8_t *in_use, uint8_t *sel_out, int *n_sel);

/* Whole .bz2 stream (compress.c:822-881 framing).  Returns output length or -1. */
int64_t orc_compress(const uint8_t *in, uint64_t n, int level, int tail_merge,
                     uint8_t *out, uint64_t out_cap);

#ifdef __cplusplus
}
#endif
#endif
