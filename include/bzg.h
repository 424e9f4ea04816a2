/* bzg.h -- C ABI of the MI355X bzip2 compression engine (libbz2_amd.so).
 *
 * The engine is the device-side replacement of the reference's per-block compression path:
 *   BZ2_compressBlock (reference compress.c:822-881) with BZ2_blockSort (blocksort.c:1534),
 *   generateMTFValues (compress.c:93), sendMTFValues (compress.c:250) and the RLE1 /
 *   block-segmentation loop copy_input_until_stop / handle_compress (bzlib.c:211-396).
 * The same library also exports the unchanged bzlib.h ABI (see include/bzlib.h); these bzg_*
 * entry points are the thin C layer under it, usable directly with device-resident buffers.
 *
 * All pointers are plain pointers; sizes are bytes.  d_* pointers are HIP device pointers on
 * the engine's current device.  `stream` is a hipStream_t (NULL = the engine's own stream).
 * Return values use the bzlib.h codes (BZ_OK, BZ_PARAM_ERROR, BZ_MEM_ERROR, BZ_OUTBUFF_FULL,
 * BZ_CONFIG_ERROR when no usable GPU is present).  The engine never calls exit().
 */
#ifndef BZG_H
#define BZG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Stream state carried between batches of one .bz2 stream. */
typedef struct {
  uint32_t combined_crc; /* running combined CRC (compress.c:827-828) */
  uint32_t blocks_done;  /* blocks emitted so far */
  uint8_t carry_byte;    /* pending high bits of an unfinished output byte */
  uint8_t carry_bits;    /* 0..7 */
  uint8_t header_done;   /* "BZh<level>" already emitted */
  uint8_t level;         /* blockSize100k, 1..9 */
} bzg_stream_state;

void bzg_stream_init(bzg_stream_state *st, int level);

/* Flags for bzg_compress_device. */
#define BZG_FLAG_END_SEGMENT 1u /* flush the pending run (FLUSH/FINISH semantics)        */
#define BZG_FLAG_TAIL_MERGE 2u  /* the last input byte arrived with FLUSH/FINISH          */
#define BZG_FLAG_TRAILER 4u     /* write the end-of-stream trailer (FINISH)              */

/* Compress a device-resident byte range as the continuation of stream `st`.
 * Without BZG_FLAG_END_SEGMENT only complete blocks are emitted and *consumed may be < n:
 * the caller re-submits input from d_in + *consumed (RUN semantics, bzlib.c:383-386).
 * The output written to d_out starts with st->carry_bits pending bits (merged), and
 * *out_bytes whole bytes are final; the unfinished last byte moves to st->carry_*.
 * Replaces: the compress half of handle_compress (bzlib.c:361-396). */
int bzg_compress_device(const void *d_in, uint64_t n, unsigned flags, bzg_stream_state *st, void *d_out,
                        uint64_t out_cap, uint64_t *out_bytes, uint64_t *consumed, void *stream);

/* Host-buffer convenience: one whole .bz2 stream (FINISH with all input, i.e. the segmentation
 * of BZ2_bzBuffToBuffCompress, bzlib.c:1309-1357).  Returns BZ_OK / BZ_OUTBUFF_FULL / ... */
int bzg_compress_host(const void *src, uint64_t n, int level, void *dst, uint64_t dst_cap, uint64_t *dst_len);

/* Host buffers, stream continuation: the same contract as bzg_compress_device with src/dst in
 * host memory (one H2D and one D2H copy).  Used by BZ2_bzCompress's staging. */
int bzg_compress_host_stream(const void *src, uint64_t n, unsigned flags, bzg_stream_state *st, void *dst,
                             uint64_t dst_cap, uint64_t *dst_len, uint64_t *consumed);

/* Worst-case output bytes for n input bytes (for sizing d_out). */
uint64_t bzg_bound(uint64_t n);

/* Per-stage entry points (host buffers), used by the parity tests to compare each stage with
 * the oracle.  Blocks are concatenated; offsets have nblocks+1 entries. */
int bzg_stage_rle1(const void *src, uint64_t n, int level, int tail_merge, uint8_t *blocks, uint64_t blocks_cap,
                   uint32_t *offsets, uint32_t *crcs, uint32_t *nblocks, uint32_t max_blocks);
int bzg_stage_bwt(const uint8_t *blocks, const uint32_t *offsets, uint32_t nblocks, uint8_t *bwt, int32_t *origptr);
/* bzg_stage_mtf: block b's nmtf[b] values at mtfv[mtf_offsets[b]] (offsets 8-aligned); mtfv
 * holds mtfv_cap values, and offsets[nblocks] + 8 * nblocks + 16 always suffice.  Returns
 * BZ_OUTBUFF_FULL (nothing written to mtfv) when mtf_offsets[nblocks] > mtfv_cap. */
int bzg_stage_mtf(const uint8_t *bwt, const uint32_t *offsets, uint32_t nblocks, uint16_t *mtfv,
                  uint64_t mtfv_cap, uint32_t *mtf_offsets, uint32_t *nmtf, uint32_t *freq);
/* BZ2_hbMakeCodeLengths (reference huffman.c:63-148) on the GPU for ntables tables: freq holds
 * kMaxAlpha (258) counts per table, alpha[t] in 2..258 of them used; lens the same layout. */
int bzg_stage_code_lengths(const uint32_t *freq, const int32_t *alpha, uint32_t ntables, int max_len, uint8_t *lens);

/* origPtr the reference assigns to one exactly periodic block w^k (SURVEY.md 8a row A5;
 * the copy-rank model of bzip2_amd/csrc/copyrank.cpp: closed form when the root has one B*
 * suffix, else a replay of the reference's divsufsort passes on the root).
 * Returns -1 on failure.  Needs no GPU. */
int32_t bzg_periodic_origptr(const uint8_t *block, int32_t n);

/* The copy rank r (origPtr = rank of rotation 0 among the p rotations of the root, times k, plus
 * r) of the block root^k that the DEVICE computes in closed form (origptr.hip: one B* offset per
 * period, or several B* offsets in pairwise different (c0, c1) buckets within the reference's
 * rank-stage budget; bzip2_amd/csrc/copyrank_cf.cpp), or -1 when the root is left to the host
 * model.  root must be primitive, p >= 2, k >= 2.  Needs no GPU (the host mirror of the rules). */
int32_t bzg_copy_rank_closed_form(const uint8_t *root, int32_t p, int32_t k);

/* BWT and origPtr of a quasi-periodic block (smallest period p <= 256 with 2p <= n not
 * dividing n, e.g. the last block of a single-repeated-byte input), computed on the host by the
 * analytic order of bzip2_amd/csrc/qsa.cpp that the GPU sort uses for such blocks (k_qsa).
 * Returns p, or 0 (nothing written) when the block is not quasi-periodic.  Needs no GPU. */
uint32_t bzg_qperiodic_bwt(const uint8_t *block, uint32_t n, uint8_t *bwt, uint32_t *origptr);

/* Timing of the last bzg_compress_device call, per stage, from HIP events (ms). */
typedef struct {
  float rle1_ms, bwt_ms, mtf_ms, code_ms, total_ms;
  uint32_t nblocks;
  uint32_t sort_iterations;
  uint64_t rle_bytes;         /* RLE1 output bytes (block bytes) */
  uint64_t sort_unsorted;     /* elements revisited by doubling iterations */
  uint64_t mtf_symbols;       /* total nMTF */
  uint32_t a5_roots;          /* periodic roots with several B* offsets (A5) */
  uint32_t a5_host;           /* of those, the ones the host model resolved (the rest: on the device) */
} bzg_stats;
/* One region of a sharded stream (the ranks of a job each hold a contiguous
 * shard of one input stream).  The global block cuts of bzlib.c:211-315 copy_input_until_stop
 * (a block ends once it holds >= nblockMAX RLE1 bytes; the pending run starts the next one)
 * depend on every byte before them, so ranks walk them in order; these two calls are the
 * per-rank part of that chain.
 *  bzg_seg_map:  RLE1 chunk map of d_in[0, n) (device memory, n <= 1.5e9), a region that starts
 *                at a chunk start of the stream (a run start, or 255 bytes into a run).  Runs
 *                on `stream` (0 = the library's own); kept until the next bzg_seg_map.
 *  bzg_seg_walk: block cuts of the mapped region when the open block already holds fill_in
 *                (< nblockMAX) RLE1 bytes at the region start: region-relative input offsets
 *                of the blocks that start inside it (ascending), the offset of the region's
 *                last chunk start and the open block's fill there.  final_region: the region
 *                ends the stream (FINISH: the last input byte never starts a block by itself,
 *                bzlib.c:276-308, 361-396).  BZ_OUTBUFF_FULL when more than max_cuts cuts exist. */
int bzg_seg_map(const void *d_in, uint64_t n, int level, void *stream);
int bzg_seg_walk(uint32_t fill_in, int final_region, uint64_t *cuts, uint32_t max_cuts, uint32_t *ncuts,
                 uint64_t *last_chunk, uint32_t *last_fill);
/* Block boundaries of an existing .bz2 stream (the prerequisite of
 * block-parallel decoding): every bit offset of d_in[0, n) (device memory) where a block-header
 * magic 0x314159265359 or the end-of-stream magic 0x177245385090 starts, ascending, as
 * out[i] = 2 * bit_offset + kind (kind 0 = block header, 1 = end of stream); bit 0 is the MSB of
 * byte 0.  Magics that occur by chance inside block data are reported too, as the reference's
 * scan reports them.  *count = the number found; BZ_OUTBUFF_FULL when it exceeds cap (out holds
 * the first cap).  Replaces the bit-serial scan of bzip2recover.c:360-395. */
int bzg_find_magics(const void *d_in, uint64_t n, uint64_t *out, uint64_t cap, uint64_t *count, void *stream);
/* GPU decompression: decode the .bz2 stream d_in[0, n) (device memory)
 * into d_out[0, out_cap) (device memory); *out_len = bytes written.  Blocks are found by the
 * magic scan and decoded in parallel (Huffman + inverse MTF, inverse BWT, un-RLE1, CRCs).
 * Returns BZ_OK for a complete stream with correct CRCs, else the code the reference's
 * BZ2_bzBuffToBuffDecompress returns for the same input (bzlib.c:1361-1410): BZ_DATA_ERROR,
 * BZ_DATA_ERROR_MAGIC, BZ_UNEXPECTED_EOF, BZ_OUTBUFF_FULL; BZ_MEM_ERROR / BZ_CONFIG_ERROR for
 * device failures.  Replaces: BZ2_bzDecompress's decode loop (decompress.c:232-…,
 * huffman.c:180-236, bzlib.c:531-677) for a whole in-memory stream. */
int bzg_decompress_device(const void *d_in, uint64_t n, void *d_out, uint64_t out_cap, uint64_t *out_len,
                          void *stream);
/* The same with host buffers (one H2D and one D2H copy); used by BZ2_bzBuffToBuffDecompress. */
int bzg_decompress_host(const void *src, uint64_t n, void *dst, uint64_t dst_cap, uint64_t *dst_len);
typedef struct {
  float total_ms;       /* device time of the last decompression */
  uint64_t blocks;      /* blocks decoded */
  uint64_t candidates;  /* block magics decoded speculatively (blocks + chance matches) */
  uint64_t out_bytes;
} bzg_decode_stats;
void bzg_last_decode_stats(bzg_decode_stats *out);
void bzg_last_stats(bzg_stats *out);

/* Release the engine's device memory (it is re-acquired on the next call). */
void bzg_release(void);

/* 1 if a HIP device is usable by the engine. */
int bzg_device_ok(void);

#ifdef __cplusplus
}
#endif
#endif
