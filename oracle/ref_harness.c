/* Test-infrastructure harness around the REFERENCE libbz2 (compiled from /root/reference by
 * oracle/Makefile into oracle/_ref/libbz2_ref.so).  It exposes the reference's internal
 * per-stage functions so that tests can pin this repo's oracle and GPU kernels stage by stage:
 *   ref_blocksort        -> BZ2_blockSort (blocksort.c:1534), BWT bytes + origPtr
 *   ref_hb_code_lengths  -> BZ2_hbMakeCodeLengths (huffman.c:63)
 * The state layout follows BZ2_bzCompressInit (bzlib.c:172-197): block = arr2 + 1 so that
 * block[-1] and block[n] exist; ptr aliases arr1; ftab is 65537 words; mtfFreq doubles as
 * divsufsort's bucket_A.  Never linked into the product. */
#include <stdlib.h>
#include <string.h>
#include "bzlib_private.h"

int ref_blocksort(const unsigned char *blk, int n, unsigned char *bwt_out)
{
   EState s;
   int i, orig;
   memset(&s, 0, sizeof(s));
   s.arr1 = (UInt32 *)calloc((size_t)n + 2, sizeof(UInt32));
   s.arr2 = (UChar *)calloc((size_t)n + 4, 1);
   s.ftab = (UInt32 *)calloc(65537, sizeof(UInt32));
   if (!s.arr1 || !s.arr2 || !s.ftab) { free(s.arr1); free(s.arr2); free(s.ftab); return -2; }
   s.ptr = s.arr1;
   s.block = s.arr2 + 1;
   memcpy(s.block, blk, (size_t)n);
   s.nblock = n;
   BZ2_blockSort(&s);
   for (i = 0; i < n; i++) bwt_out[i] = (unsigned char)s.ptr[i];
   orig = s.origPtr;
   free(s.arr1); free(s.arr2); free(s.ftab);
   return orig;
}

void ref_hb_code_lengths(int *len, int *freq, int alphaSize, int maxLen)
{
   BZ2_hbMakeCodeLengths(len, freq, alphaSize, maxLen);
}

/* CRC table identity check: the reference table is BZ2_crc32Table (crctable.c). */
unsigned int ref_crc_table_entry(int i) { return BZ2_crc32Table[i & 255]; }
