/* bz_oracle.c -- TEST INFRASTRUCTURE ONLY (see bz_oracle.h).
 *
 * A deliberately simple, single-threaded restatement of the reference's compression path.
 * Each function names the reference lines whose behaviour it restates.  Nothing here is
 * tuned for speed: it is the checker the HIP kernels are compared against.
 */
#include "bz_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ CRC (A2) */
/* MSB-first CRC-32 with polynomial 0x04C11DB7, init ~0, final ~ (bzlib_private.h:187-202).
 * The table is generated from the polynomial rather than copied from crctable.c; the tests
 * compare it entry by entry with the reference table. */
static uint32_t g_crc[256];
static int g_crc_ready = 0;

static void crc_init(void)
{
  if (g_crc_ready) return;
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t r = i << 24;
    for (int b = 0; b < 8; b++) r = (r & 0x80000000u) ? (r << 1) ^ 0x04C11DB7u : (r << 1);
    g_crc[i] = r;
  }
  g_crc_ready = 1;
}

uint32_t orc_crc_table(int i)
{
  crc_init();
  return g_crc[i & 255];
}

uint32_t orc_crc_update(uint32_t crc, const uint8_t *p, uint64_t n)
{
  crc_init();
  for (uint64_t i = 0; i < n; i++) crc = (crc << 8) ^ g_crc[(crc >> 24) ^ p[i]];
  return crc;
}

/* ------------------------------------------------------------------ RLE1 (A1) */
/* Restates copy_input_until_stop (bzlib.c:211-315) and the block-cut rule of handle_compress
 * (bzlib.c:381-386).  A byte is only consumed while the block holds fewer than nblockMAX
 * (= 100000*level - 19, bzlib.c:190) bytes; a pending run carries into the next block. */
typedef struct {
  uint8_t *blocks;
  uint64_t cap, nblk_bytes;   /* bytes written to the current block */
  uint64_t base;              /* offset of the current block in blocks[] */
  uint32_t crc;
  int overflow;
} rle_state;

static void rle_emit(rle_state *s, uint8_t c)
{
  if (s->base + s->nblk_bytes >= s->cap) { s->overflow = 1; return; }
  s->blocks[s->base + s->nblk_bytes++] = c;
}

static void rle_flush_run(rle_state *s, uint32_t ch, uint32_t len)
{
  /* bzlib.c:237-257: runs of 1..3 are copied, runs of 4..255 become 4 copies + (len-4). */
  uint32_t copies = len < 4 ? len : 4;
  for (uint32_t k = 0; k < copies; k++) rle_emit(s, (uint8_t)ch);
  if (len >= 4) rle_emit(s, (uint8_t)(len - 4));
  for (uint32_t k = 0; k < len; k++) s->crc = (s->crc << 8) ^ g_crc[(s->crc >> 24) ^ ch];
}

int64_t orc_rle1(const uint8_t *in, uint64_t n, int level, int tail_merge,
                 uint8_t *blocks, uint64_t blocks_cap,
                 uint64_t *blk_off, uint32_t *blk_crc, int64_t max_blocks)
{
  crc_init();
  rle_state s = {blocks, blocks_cap, 0, 0, 0xffffffffu, 0};
  const uint64_t nblock_max = 100000u * (uint64_t)level - 19u;
  uint32_t ch = 256, len = 0;   /* init_RL (bzlib.c:134-138) */
  uint64_t i = 0;
  int64_t nb = 0;
  if (n == 0) { blk_off[0] = 0; return 0; }

  for (;;) {
    while (s.nblk_bytes < nblock_max && i < n) {
      uint32_t z = in[i++];
      if (z != ch && len == 1) {            /* bzlib.c:231-235 */
        s.crc = (s.crc << 8) ^ g_crc[(s.crc >> 24) ^ ch];
        rle_emit(&s, (uint8_t)ch);
        ch = z;
      } else if (z != ch || len == 255) {   /* bzlib.c:236-259 */
        if (len != 0) rle_flush_run(&s, ch, len);
        ch = z;
        len = 1;
      } else {
        len++;
      }
    }
    int input_done = (i == n);
    int cut_full = (s.nblk_bytes >= nblock_max);
    if (input_done && (tail_merge || !cut_full)) {
      /* FINISH: pending run flushed into the current block (bzlib.c:276-308). */
      rle_flush_run(&s, ch, len);
      len = 0;
    }
    if (nb >= max_blocks) return -1;
    blk_off[nb] = s.base;
    blk_crc[nb] = ~s.crc;
    nb++;
    s.base += s.nblk_bytes;
    s.nblk_bytes = 0;
    s.crc = 0xffffffffu;
    if (input_done && len == 0) break;
    /* RUN mode: a full block was cut exactly at end of input; the pending run alone forms
     * the last block (bzlib.c:383-386 then the FINISH call's flush). */
    if (input_done) {
      rle_flush_run(&s, ch, len);
      len = 0;
      if (nb >= max_blocks) return -1;
      blk_off[nb] = s.base;
      blk_crc[nb] = ~s.crc;
      nb++;
      s.base += s.nblk_bytes;
      s.nblk_bytes = 0;
      break;
    }
  }
  blk_off[nb] = s.base;
  return s.overflow ? -1 : nb;
}

/* ------------------------------------------------------------------ BWT (A4/A5) */
static orc_resolver_fn g_resolver = 0;
void orc_set_resolver(orc_resolver_fn fn) { g_resolver = fn; }

/* Smallest p dividing n with blk[i] == blk[(i+p) mod n] for all i (KMP failure function). */
static int primitive_period(const uint8_t *t, int n)
{
  int *f = (int *)malloc(sizeof(int) * ((size_t)n + 1));
  f[0] = -1;
  for (int i = 1; i <= n; i++) {
    int k = f[i - 1];
    while (k >= 0 && t[k] != t[i - 1]) k = f[k];
    f[i] = k + 1;
  }
  int p = n - f[n];
  free(f);
  return (n % p == 0) ? p : n;
}

/* Cyclic suffix array of an aperiodic string by prefix doubling with counting sorts.  Every
 * rotation is distinct, so the order is unique and equals the reference's
 * (parity fact 3). */
static void cyclic_sa(const uint8_t *t, int n, int *sa)
{
  int *rk = (int *)malloc(sizeof(int) * (size_t)n);
  int *tmp = (int *)malloc(sizeof(int) * (size_t)n);
  int *cnt = (int *)malloc(sizeof(int) * ((size_t)(n > 256 ? n : 256) + 1));
  int classes;
  memset(cnt, 0, sizeof(int) * 257);
  for (int i = 0; i < n; i++) cnt[t[i] + 1]++;
  for (int c = 0; c < 256; c++) cnt[c + 1] += cnt[c];
  for (int i = 0; i < n; i++) sa[cnt[t[i]]++] = i;
  rk[sa[0]] = 0;
  classes = 1;
  for (int i = 1; i < n; i++) {
    if (t[sa[i]] != t[sa[i - 1]]) classes++;
    rk[sa[i]] = classes - 1;
  }
  for (int h = 1; classes < n && h < n; h <<= 1) {
    /* order by (rk[i], rk[i+h]): counting sort on the first key of i-h. */
    for (int i = 0; i < n; i++) { int j = sa[i] - h; tmp[i] = j < 0 ? j + n : j; }
    memset(cnt, 0, sizeof(int) * ((size_t)classes + 1));
    for (int i = 0; i < n; i++) cnt[rk[tmp[i]] + 1]++;
    for (int c = 0; c < classes; c++) cnt[c + 1] += cnt[c];
    for (int i = 0; i < n; i++) sa[cnt[rk[tmp[i]]]++] = tmp[i];
    tmp[sa[0]] = 0;
    classes = 1;
    for (int i = 1; i < n; i++) {
      int a = sa[i], b = sa[i - 1];
      int a2 = a + h >= n ? a + h - n : a + h, b2 = b + h >= n ? b + h - n : b + h;
      if (rk[a] != rk[b] || rk[a2] != rk[b2]) classes++;
      tmp[a] = classes - 1;
    }
    memcpy(rk, tmp, sizeof(int) * (size_t)n);
  }
  free(rk); free(tmp); free(cnt);
}

int orc_bwt(const uint8_t *blk, int n, uint8_t *bwt, int *period_out)
{
  if (n <= 0) return -1;
  if (n == 1) { bwt[0] = blk[0]; if (period_out) *period_out = 1; return 0; }
  int p = primitive_period(blk, n);
  if (period_out) *period_out = p;
  int *sa = (int *)malloc(sizeof(int) * (size_t)p);
  cyclic_sa(blk, p, sa);
  int k = n / p, rank0 = 0;
  for (int j = 0; j < p; j++) {
    uint8_t c = blk[sa[j] == 0 ? p - 1 : sa[j] - 1];
    for (int r = 0; r < k; r++) bwt[j * k + r] = c;
    if (sa[j] == 0) rank0 = j;
  }
  free(sa);
  if (k == 1) return rank0;
  if (p == 1) return 0;   /* single-symbol block: no B* suffix, origPtr 0 (blocksort.c:1349) */
  /* Exactly periodic block: identical rotations tie; the reference's order among them is
   * delegated (A5). */
  if (!g_resolver) return -1;
  uint8_t *scratch = (uint8_t *)malloc((size_t)n);
  int orig = g_resolver(blk, n, scratch);
  free(scratch);
  return orig;
}

/* ------------------------------------------------------------------ MTF (A6) */
/* generateMTFValues (compress.c:93-229): list starts as the in-use bytes ascending; a run
 * of z zeros is written as bijective base-2 digits RUNA=0 / RUNB=1, least significant first;
 * a non-zero rank j is written as j+1; EOB = nInUse+1 closes the block. */
int orc_mtf(const uint8_t *bwt, int n, uint16_t *mtfv, int32_t *freq, int *n_in_use)
{
  uint8_t used[256] = {0}, list[256];
  int nu = 0, out = 0;
  uint32_t zrun = 0;
  for (int i = 0; i < n; i++) used[bwt[i]] = 1;
  for (int c = 0; c < 256; c++) if (used[c]) list[nu++] = (uint8_t)c;
  for (int v = 0; v < 258; v++) freq[v] = 0;
  for (int i = 0; i <= n; i++) {
    int pos = 0;
    if (i < n) {
      while (list[pos] != bwt[i]) pos++;
      if (pos == 0) { zrun++; continue; }
    }
    while (zrun > 0) {
      zrun--;
      uint16_t d = (uint16_t)(zrun & 1);
      mtfv[out++] = d;
      freq[d]++;
      zrun >>= 1;
    }
    if (i == n) break;
    uint8_t c = list[pos];
    memmove(list + 1, list, (size_t)pos);
    list[0] = c;
    mtfv[out++] = (uint16_t)(pos + 1);
    freq[pos + 1]++;
  }
  mtfv[out++] = (uint16_t)(nu + 1);
  freq[nu + 1] = 1;
  *n_in_use = nu;
  return out;
}

/* ------------------------------------------------------------------ Huffman (A8) */
/* BZ2_hbMakeCodeLengths (huffman.c:63-148).  A node weight carries the subtree depth in its
 * low 8 bits, so equal frequencies are broken by depth; heap moves compare with strict '<'.
 * If a code exceeds max_len every leaf weight is halved (1 + w/2) and the tree rebuilt. */
void orc_code_lengths(int32_t *len, const int32_t *freq, int alpha, int max_len)
{
  int32_t heap[260 + 2], weight[258 * 2], parent[258 * 2];
  for (int i = 0; i < alpha; i++) weight[i + 1] = (freq[i] == 0 ? 1 : freq[i]) << 8;
  for (;;) {
    int nodes = alpha, nheap = 0;
    heap[0] = 0; weight[0] = 0; parent[0] = -2;
    for (int i = 1; i <= alpha; i++) {
      parent[i] = -1;
      heap[++nheap] = i;
      int z = nheap, item = heap[z];
      while (weight[item] < weight[heap[z >> 1]]) { heap[z] = heap[z >> 1]; z >>= 1; }
      heap[z] = item;
    }
    while (nheap > 1) {
      int pick[2];
      for (int k = 0; k < 2; k++) {
        pick[k] = heap[1];
        heap[1] = heap[nheap--];
        int z = 1, item = heap[1];
        for (;;) {
          int y = z << 1;
          if (y > nheap) break;
          if (y < nheap && weight[heap[y + 1]] < weight[heap[y]]) y++;
          if (weight[item] < weight[heap[y]]) break;
          heap[z] = heap[y];
          z = y;
        }
        heap[z] = item;
      }
      nodes++;
      parent[pick[0]] = parent[pick[1]] = nodes;
      int32_t w0 = weight[pick[0]], w1 = weight[pick[1]];
      int32_t d0 = w0 & 0xff, d1 = w1 & 0xff;
      weight[nodes] = (int32_t)(((uint32_t)w0 & 0xffffff00u) + ((uint32_t)w1 & 0xffffff00u)) |
                      (1 + (d0 > d1 ? d0 : d1));
      parent[nodes] = -1;
      heap[++nheap] = nodes;
      int z = nheap, item = heap[z];
      while (weight[item] < weight[heap[z >> 1]]) { heap[z] = heap[z >> 1]; z >>= 1; }
      heap[z] = item;
    }
    int too_long = 0;
    for (int i = 1; i <= alpha; i++) {
      int d = 0, k = i;
      while (parent[k] >= 0) { k = parent[k]; d++; }
      len[i - 1] = d;
      if (d > max_len) too_long = 1;
    }
    if (!too_long) return;
    for (int i = 1; i <= alpha; i++) weight[i] = (1 + ((weight[i] >> 8) / 2)) << 8;
  }
}

/* ------------------------------------------------------------------ bit writer */
void orc_put(orc_bits *w, int nbits, uint32_t v)
{
  for (int b = nbits - 1; b >= 0; b--) {
    uint64_t pos = w->nbits++;
    if ((pos >> 3) >= w->cap) continue;
    if ((v >> b) & 1u) w->buf[pos >> 3] |= (uint8_t)(0x80u >> (pos & 7));
    else w->buf[pos >> 3] &= (uint8_t)~(0x80u >> (pos & 7));
  }
}

/* ------------------------------------------------------------------ tables (A7) */
int orc_send_mtf(orc_bits *w, const uint16_t *mtfv, int n_mtf, const int32_t *freq,
                 int n_in_use, const uint8_t *in_use, uint8_t *sel_out, int *n_sel)
{
  enum { G = 50, MAXSEL = 18002 };
  static int32_t len[6][258], rfreq[6][258], code[6][258];
  static uint8_t sel[MAXSEL];
  int alpha = n_in_use + 2, ng, nsel = 0;
  /* compress.c:266-270 */
  ng = n_mtf < 200 ? 2 : n_mtf < 600 ? 3 : n_mtf < 1200 ? 4 : n_mtf < 2400 ? 5 : 6;

  /* Initial tables: contiguous symbol ranges of roughly equal frequency (compress.c:276-319). */
  for (int t = 0; t < ng; t++) for (int v = 0; v < alpha; v++) len[t][v] = 15;
  {
    int part = ng, rem = n_mtf, gs = 0;
    while (part > 0) {
      int target = rem / part, ge = gs - 1, acc = 0;
      while (acc < target && ge < alpha - 1) acc += freq[++ge];
      if (ge > gs && part != ng && part != 1 && ((ng - part) % 2 == 1)) acc -= freq[ge--];
      for (int v = gs; v <= ge; v++) len[part - 1][v] = 0;
      part--;
      gs = ge + 1;
      rem -= acc;
    }
  }

  /* Four refinement passes (compress.c:324-561). */
  for (int it = 0; it < 4; it++) {
    memset(rfreq, 0, sizeof(rfreq));
    nsel = 0;
    for (int gs = 0; gs < n_mtf; gs += G) {
      int ge = gs + G < n_mtf ? gs + G : n_mtf;
      int cost[6] = {0, 0, 0, 0, 0, 0};
      for (int i = gs; i < ge; i++) for (int t = 0; t < ng; t++) cost[t] += len[t][mtfv[i]];
      int bt = 0;
      for (int t = 1; t < ng; t++) if (cost[t] < cost[bt]) bt = t;
      sel[nsel++] = (uint8_t)bt;
      for (int i = gs; i < ge; i++) rfreq[bt][mtfv[i]]++;
    }
    for (int t = 0; t < ng; t++) orc_code_lengths(len[t], rfreq[t], alpha, 17);
  }

  /* Canonical codes (compress.c:634-651, huffman.c:152-166). */
  for (int t = 0; t < ng; t++) {
    int mn = 32, mx = 0;
    for (int v = 0; v < alpha; v++) { if (len[t][v] > mx) mx = len[t][v]; if (len[t][v] < mn) mn = len[t][v]; }
    int c = 0;
    for (int l = mn; l <= mx; l++) {
      for (int v = 0; v < alpha; v++) if (len[t][v] == l) code[t][v] = c++;
      c <<= 1;
    }
  }

  /* Symbol map: 16-bit summary then one 16-bit row per used range (compress.c:654-675). */
  {
    uint32_t top = 0;
    for (int i = 0; i < 16; i++) {
      int any = 0;
      for (int j = 0; j < 16; j++) any |= in_use[i * 16 + j];
      top = (top << 1) | (uint32_t)(any != 0);
    }
    orc_put(w, 16, top);
    for (int i = 0; i < 16; i++) {
      if (!(top & (0x8000u >> i))) continue;
      uint32_t row = 0;
      for (int j = 0; j < 16; j++) row = (row << 1) | (uint32_t)(in_use[i * 16 + j] != 0);
      orc_put(w, 16, row);
    }
  }

  /* Selectors, move-to-front coded in unary (compress.c:573-631, 680-689). */
  orc_put(w, 3, (uint32_t)ng);
  orc_put(w, 15, (uint32_t)nsel);
  {
    uint8_t order[6] = {0, 1, 2, 3, 4, 5};
    for (int i = 0; i < nsel; i++) {
      int j = 0;
      while (order[j] != sel[i]) j++;
      for (int k = j; k > 0; k--) order[k] = order[k - 1];
      order[0] = sel[i];
      orc_put(w, j + 1, (1u << (j + 1)) - 2u);
    }
  }

  /* Code lengths, delta coded (compress.c:694-706). */
  for (int t = 0; t < ng; t++) {
    int cur = len[t][0];
    orc_put(w, 5, (uint32_t)cur);
    for (int v = 0; v < alpha; v++) {
      while (cur < len[t][v]) { orc_put(w, 2, 2); cur++; }
      while (cur > len[t][v]) { orc_put(w, 2, 3); cur--; }
      orc_put(w, 1, 0);
    }
  }

  /* Payload (compress.c:713-812). */
  for (int g = 0, gs = 0; gs < n_mtf; g++, gs += G) {
    int ge = gs + G < n_mtf ? gs + G : n_mtf, t = sel[g];
    for (int i = gs; i < ge; i++) orc_put(w, len[t][mtfv[i]], (uint32_t)code[t][mtfv[i]]);
  }
  if (sel_out) memcpy(sel_out, sel, (size_t)nsel);
  if (n_sel) *n_sel = nsel;
  return 0;
}

/* ------------------------------------------------------------------ stream (A3) */
/* BZ2_compressBlock (compress.c:822-881): "BZh"+level, then per block the 48-bit magic
 * 0x314159265359, block CRC, a zero randomised bit, 24-bit origPtr and the payload; the
 * stream ends with 0x177245385090, the combined CRC, and zero bits to a byte boundary. */
int64_t orc_compress(const uint8_t *in, uint64_t n, int level, int tail_merge,
                     uint8_t *out, uint64_t out_cap)
{
  uint64_t cap = n + n / 4 + 64;
  uint8_t *blocks = (uint8_t *)malloc(cap);
  int64_t maxb = (int64_t)(n / 90000 + 4);
  uint64_t *off = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(maxb + 1));
  uint32_t *crc = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)maxb);
  int64_t nb = orc_rle1(in, n, level, tail_merge, blocks, cap, off, crc, maxb);
  if (nb < 0) { free(blocks); free(off); free(crc); return -1; }

  memset(out, 0, out_cap);
  orc_bits w = {out, out_cap, 0};
  orc_put(&w, 8, 'B'); orc_put(&w, 8, 'Z'); orc_put(&w, 8, 'h'); orc_put(&w, 8, (uint32_t)('0' + level));
  uint32_t combined = 0;
  int64_t rc = 0;
  for (int64_t b = 0; b < nb && rc == 0; b++) {
    int len = (int)(off[b + 1] - off[b]);
    const uint8_t *blk = blocks + off[b];
    uint8_t *bwt = (uint8_t *)malloc((size_t)len);
    uint16_t *mtfv = (uint16_t *)malloc(sizeof(uint16_t) * ((size_t)len + 2));
    int32_t freq[258];
    uint8_t used[256] = {0};
    int nu;
    for (int i = 0; i < len; i++) used[blk[i]] = 1;
    int orig = orc_bwt(blk, len, bwt, NULL);
    if (orig < 0) rc = -1;
    int nmtf = orc_mtf(bwt, len, mtfv, freq, &nu);
    combined = ((combined << 1) | (combined >> 31)) ^ crc[b];
    orc_put(&w, 24, 0x314159); orc_put(&w, 24, 0x265359);
    orc_put(&w, 16, crc[b] >> 16); orc_put(&w, 16, crc[b] & 0xffff);
    orc_put(&w, 1, 0);
    orc_put(&w, 24, (uint32_t)orig);
    orc_send_mtf(&w, mtfv, nmtf, freq, nu, used, NULL, NULL);
    free(bwt); free(mtfv);
  }
  orc_put(&w, 24, 0x177245); orc_put(&w, 24, 0x385090);
  orc_put(&w, 16, combined >> 16); orc_put(&w, 16, combined & 0xffff);
  free(blocks); free(off); free(crc);
  if (rc) return -1;
  uint64_t bytes = (w.nbits + 7) >> 3;
  return bytes > out_cap ? -1 : (int64_t)bytes;
}
