// decode.cpp -- resumable CPU decoder for the .bz2 format (BZ2_bzDecompressInit /
// BZ2_bzDecompress / BZ2_bzDecompressEnd).
//
// Decompression is not on the accelerated path (SURVEY.md section 8f row 2 lists it as later
// work); this decoder exists so that the library is a complete drop-in.  It is a plain
// state machine that suspends whenever the next field or Huffman symbol needs more input
// bits than are available, so it accepts input in arbitrary pieces and consumes input only
// up to the last bit it used (concatenated streams and BZ2_bzReadGetUnused keep working).
// Randomised blocks (written only by bzip2 < 0.9.5) are decoded as the reference does: every
// byte of the inverse BWT walk is XORed with the format's random mask before un-RLE1
// (bzlib_private.h:163-179, bzlib.c:535-581).
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "decode.h"

namespace {

const int32_t kRNums[512] = {
#include "rnums.inc"
};

uint32_t g_crc[256];
bool g_crc_ok = false;
void crc_init() {
  if (g_crc_ok) return;
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t r = i << 24;
    for (int k = 0; k < 8; k++) r = (r & 0x80000000u) ? (r << 1) ^ 0x04C11DB7u : (r << 1);
    g_crc[i] = r;
  }
  g_crc_ok = true;
}

enum Phase {
  kMagic, kBlockHdr, kBlockCrc, kRandBit, kOrigPtr, kMap16, kMapRows, kGroupsSel, kSelectors, kTables,
  kSymbols, kOutput, kTrailerCrc, kDone, kError
};

struct DState {
  bz_stream* strm;
  int verbosity, small;
  Phase ph;
  uint64_t bb;
  int bl;
  int level;
  uint32_t stored_bcrc, comb_crc;
  int32_t origptr;
  bool randomised;
  uint32_t map16;
  int map_i;
  uint8_t seq2byte[256];
  int nuse;
  int ngroups, nsel, sel_i, sel_j;
  uint8_t selector[18002 + 8];
  int tab_t, tab_v, tab_cur, tab_state;
  uint8_t len[6][258];
  int32_t first[6][22], count[6][22], offs[6][22];
  uint16_t perm[6][258];
  int minlen[6], maxlen[6];
  int group_no, group_pos, cur;
  uint8_t mtf[256];
  uint32_t cftab[257];
  uint32_t es, es_n;
  bool in_run;
  std::vector<uint32_t> tt;
  int32_t nblock;
  std::vector<uint8_t> out;
  size_t out_pos;
  bool stream_end_pending;
};

// Bit supply: pulls whole bytes from the caller's input only when a field needs them.
bool need(DState* s, int n) {
  bz_stream* z = s->strm;
  while (s->bl < n) {
    if (z->avail_in == 0) return false;
    s->bb = (s->bb << 8) | (uint8_t)*z->next_in;
    s->bl += 8;
    z->next_in++;
    z->avail_in--;
    if (++z->total_in_lo32 == 0) z->total_in_hi32++;
  }
  return true;
}
uint32_t take(DState* s, int n) {
  s->bl -= n;
  return (uint32_t)(s->bb >> s->bl) & (n == 32 ? 0xffffffffu : ((1u << n) - 1u));
}
// fills as many whole bytes as possible, up to `upto` buffered bits
void fill(DState* s, int upto) {
  bz_stream* z = s->strm;
  while (s->bl + 8 <= upto && z->avail_in > 0) {
    s->bb = (s->bb << 8) | (uint8_t)*z->next_in;
    s->bl += 8;
    z->next_in++;
    z->avail_in--;
    if (++z->total_in_lo32 == 0) z->total_in_hi32++;
  }
}

bool build_tables(DState* s) {
  const int alpha = s->nuse + 2;
  for (int t = 0; t < s->ngroups; t++) {
    int mn = 32, mx = 0;
    for (int v = 0; v < alpha; v++) {
      mn = s->len[t][v] < mn ? s->len[t][v] : mn;
      mx = s->len[t][v] > mx ? s->len[t][v] : mx;
    }
    s->minlen[t] = mn;
    s->maxlen[t] = mx;
    int32_t code = 0, idx = 0;
    for (int l = mn; l <= mx; l++) {
      s->first[t][l] = code;
      s->offs[t][l] = idx;
      int c = 0;
      for (int v = 0; v < alpha; v++)
        if (s->len[t][v] == l) s->perm[t][idx + c++] = (uint16_t)v;
      s->count[t][l] = c;
      idx += c;
      code = (code + c) << 1;
    }
  }
  return true;
}

// Finishes a block: inverse BWT, RLE1 decode, CRC check.  Appends to s->out.
bool finish_block(DState* s) {
  const int32_t n = s->nblock;
  if (s->origptr < 0 || s->origptr >= n) return false;
  uint32_t c[257];
  c[0] = 0;
  for (int i = 0; i < 256; i++) c[i + 1] = c[i] + s->cftab[i];
  uint32_t* tt = s->tt.data();
  for (int32_t i = 0; i < n; i++) {
    const uint32_t ch = tt[i] & 0xffu;
    tt[c[ch]++] |= (uint32_t)i << 8;
  }
  uint32_t pos = tt[s->origptr] >> 8;
  uint32_t crc = 0xffffffffu;
  int run = 0, last = -1;
  const size_t base = s->out.size();
  s->out.reserve(base + (size_t)n + 64);
  int32_t r_togo = 0, r_pos = 0;  // the random mask of a randomised block, one step per walk byte
  for (int32_t k = 0; k < n; k++) {
    pos = tt[pos];
    uint32_t ch = pos & 0xffu;
    pos >>= 8;
    if (s->randomised) {
      if (r_togo == 0) {
        r_togo = kRNums[r_pos];
        r_pos = (r_pos + 1) & 511;
      }
      r_togo--;
      ch ^= r_togo == 1 ? 1u : 0u;
    }
    if (run == 4) {
      for (uint32_t r = 0; r < ch; r++) {
        s->out.push_back((uint8_t)last);
        crc = (crc << 8) ^ g_crc[(crc >> 24) ^ (uint32_t)last];
      }
      run = 0;
      last = -1;
      continue;
    }
    if ((int)ch == last) run++;
    else {
      run = 1;
      last = (int)ch;
    }
    s->out.push_back((uint8_t)ch);
    crc = (crc << 8) ^ g_crc[(crc >> 24) ^ ch];
  }
  crc = ~crc;
  if (crc != s->stored_bcrc) return false;
  s->comb_crc = ((s->comb_crc << 1) | (s->comb_crc >> 31)) ^ crc;
  return true;
}

// Runs the state machine as far as the input allows.  Returns BZ_OK, BZ_STREAM_END-ready
// (via stream_end_pending), or an error code.
int advance(DState* s) {
  for (;;) {
    switch (s->ph) {
      case kMagic: {
        if (!need(s, 32)) return BZ_OK;
        const uint32_t v = take(s, 32);
        if ((v >> 8) != 0x425a68u) return BZ_DATA_ERROR_MAGIC;
        const int lv = (int)(v & 0xff) - '0';
        if (lv < 1 || lv > 9) return BZ_DATA_ERROR_MAGIC;
        s->level = lv;
        s->ph = kBlockHdr;
        break;
      }
      case kBlockHdr: {
        if (!need(s, 48)) return BZ_OK;
        const uint32_t hi = take(s, 24);
        const uint32_t lo = take(s, 24);
        if (hi == 0x314159u) {
          if (lo != 0x265359u) return BZ_DATA_ERROR;
          s->ph = kBlockCrc;
        } else {
          if (lo != 0x385090u) return BZ_DATA_ERROR;
          s->ph = kTrailerCrc;
        }
        break;
      }
      case kBlockCrc:
        if (!need(s, 32)) return BZ_OK;
        s->stored_bcrc = take(s, 32);
        s->ph = kRandBit;
        break;
      case kRandBit:
        if (!need(s, 1)) return BZ_OK;
        s->randomised = take(s, 1) != 0;  // randomised block (pre-0.9.5 encoders)
        s->ph = kOrigPtr;
        break;
      case kOrigPtr:
        if (!need(s, 24)) return BZ_OK;
        s->origptr = (int32_t)take(s, 24);
        if (s->origptr > 100000 * s->level) return BZ_DATA_ERROR;
        s->ph = kMap16;
        break;
      case kMap16:
        if (!need(s, 16)) return BZ_OK;
        s->map16 = take(s, 16);
        s->map_i = 0;
        s->nuse = 0;
        s->ph = kMapRows;
        break;
      case kMapRows:
        while (s->map_i < 16) {
          if (s->map16 & (0x8000u >> s->map_i)) {
            if (!need(s, 16)) return BZ_OK;
            const uint32_t row = take(s, 16);
            for (int j = 0; j < 16; j++)
              if (row & (0x8000u >> j)) s->seq2byte[s->nuse++] = (uint8_t)(s->map_i * 16 + j);
          }
          s->map_i++;
        }
        if (s->nuse == 0) return BZ_DATA_ERROR;
        s->ph = kGroupsSel;
        break;
      case kGroupsSel: {
        if (!need(s, 18)) return BZ_OK;
        const uint32_t v = take(s, 18);
        s->ngroups = (int)(v >> 15);
        s->nsel = (int)(v & 0x7fffu);
        if (s->ngroups < 2 || s->ngroups > 6) return BZ_DATA_ERROR;
        if (s->nsel < 1 || s->nsel > 18002) return BZ_DATA_ERROR;
        s->sel_i = 0;
        s->sel_j = 0;
        s->ph = kSelectors;
        break;
      }
      case kSelectors:
        while (s->sel_i < s->nsel) {
          if (!need(s, 1)) return BZ_OK;
          if (take(s, 1)) {
            if (++s->sel_j >= s->ngroups) return BZ_DATA_ERROR;
          } else {
            s->selector[s->sel_i++] = (uint8_t)s->sel_j;
            s->sel_j = 0;
          }
        }
        {  // undo the selector MTF
          uint8_t order[6] = {0, 1, 2, 3, 4, 5};
          for (int i = 0; i < s->nsel; i++) {
            const int j = s->selector[i];
            const uint8_t t = order[j];
            for (int k = j; k > 0; k--) order[k] = order[k - 1];
            order[0] = t;
            s->selector[i] = t;
          }
        }
        s->tab_t = 0;
        s->tab_v = -1;
        s->ph = kTables;
        break;
      case kTables: {
        const int alpha = s->nuse + 2;
        while (s->tab_t < s->ngroups) {
          if (s->tab_v < 0) {
            if (!need(s, 5)) return BZ_OK;
            s->tab_cur = (int)take(s, 5);
            s->tab_v = 0;
          }
          while (s->tab_v < alpha) {
            if (s->tab_cur < 1 || s->tab_cur > 20) return BZ_DATA_ERROR;
            if (!need(s, 1)) return BZ_OK;
            if ((s->bb >> (s->bl - 1)) & 1u) {
              if (!need(s, 2)) return BZ_OK;
              const uint32_t two = take(s, 2);
              s->tab_cur += (two & 1u) ? -1 : 1;
            } else {
              take(s, 1);
              s->len[s->tab_t][s->tab_v++] = (uint8_t)s->tab_cur;
            }
          }
          s->tab_t++;
          s->tab_v = -1;
        }
        build_tables(s);
        for (int i = 0; i < s->nuse; i++) s->mtf[i] = (uint8_t)i;
        for (int i = 0; i < 256; i++) s->cftab[i] = 0;
        s->tt.resize((size_t)s->level * 100000);
        s->nblock = 0;
        s->group_no = -1;
        s->group_pos = 0;
        s->in_run = false;
        s->es = 0;
        s->es_n = 1;
        s->ph = kSymbols;
        break;
      }
      case kSymbols: {
        const int eob = s->nuse + 1;
        const int32_t cap = s->level * 100000;
        for (;;) {
          if (s->group_pos == 0) {
            if (++s->group_no >= s->nsel) return BZ_DATA_ERROR;
            s->group_pos = 50;
            s->cur = s->selector[s->group_no];
          }
          const int t = s->cur;
          fill(s, 56);
          int zn = s->minlen[t], sym = -1;
          for (; zn <= s->maxlen[t]; zn++) {
            if (zn > s->bl) break;
            const uint32_t zv = (uint32_t)(s->bb >> (s->bl - zn)) & ((1u << zn) - 1u);
            const uint32_t d = zv - (uint32_t)s->first[t][zn];
            if (d < (uint32_t)s->count[t][zn]) {
              sym = s->perm[t][s->offs[t][zn] + (int)d];
              break;
            }
          }
          if (sym < 0) {
            if (zn <= s->maxlen[t] && s->strm->avail_in == 0) {
              // not enough bits yet: undo an untouched group advance and wait for input
              if (s->group_pos == 50) {
                s->group_no--;
                s->group_pos = 0;
              }
              return BZ_OK;
            }
            return BZ_DATA_ERROR;
          }
          s->bl -= zn;
          s->group_pos--;
          if (sym <= 1) {  // RUNA / RUNB
            if (!s->in_run) {
              s->in_run = true;
              s->es = 0;
              s->es_n = 1;
            }
            if (s->es_n > (1u << 21)) return BZ_DATA_ERROR;
            s->es += (uint32_t)(sym + 1) * s->es_n;
            s->es_n <<= 1;
            continue;
          }
          if (s->in_run) {
            const uint8_t b = s->seq2byte[s->mtf[0]];
            if ((int64_t)s->nblock + s->es > cap) return BZ_DATA_ERROR;
            for (uint32_t r = 0; r < s->es; r++) s->tt[s->nblock++] = b;
            s->cftab[b] += s->es;
            s->in_run = false;
          }
          if (sym == eob) break;
          const int j = sym - 1;
          if (j >= s->nuse) return BZ_DATA_ERROR;
          const uint8_t m = s->mtf[j];
          std::memmove(s->mtf + 1, s->mtf, (size_t)j);
          s->mtf[0] = m;
          if (s->nblock >= cap) return BZ_DATA_ERROR;
          const uint8_t b = s->seq2byte[m];
          s->tt[s->nblock++] = b;
          s->cftab[b]++;
        }
        if (!finish_block(s)) return BZ_DATA_ERROR;
        s->ph = kBlockHdr;
        return BZ_OK;  // let the caller drain this block before decoding the next
      }
      case kTrailerCrc: {
        if (!need(s, 32)) return BZ_OK;
        const uint32_t c = take(s, 32);
        if (c != s->comb_crc) return BZ_DATA_ERROR;
        s->bl = 0;  // discard the byte padding
        s->ph = kDone;
        s->stream_end_pending = true;
        return BZ_OK;
      }
      default:
        return BZ_OK;
    }
  }
}

void drain(DState* s) {
  bz_stream* z = s->strm;
  const size_t left = s->out.size() - s->out_pos;
  const size_t cnt = left < z->avail_out ? left : z->avail_out;
  if (cnt) {
    std::memcpy(z->next_out, s->out.data() + s->out_pos, cnt);
    z->next_out += cnt;
    z->avail_out -= (unsigned)cnt;
    const unsigned t = z->total_out_lo32 + (unsigned)cnt;
    if (t < z->total_out_lo32) z->total_out_hi32++;
    z->total_out_lo32 = t;
    s->out_pos += cnt;
  }
  if (s->out_pos == s->out.size()) {
    s->out.clear();
    s->out_pos = 0;
  }
}

void* dflt_alloc(void*, int items, int size) { return std::malloc((size_t)items * (size_t)size); }
void dflt_free(void*, void* p) { std::free(p); }

}  // namespace

extern "C" {

int BZ2_bzDecompressInit(bz_stream* strm, int verbosity, int small) {
  if (strm == nullptr || (small != 0 && small != 1) || verbosity < 0 || verbosity > 4) return BZ_PARAM_ERROR;
  crc_init();
  if (strm->bzalloc == nullptr) strm->bzalloc = dflt_alloc;
  if (strm->bzfree == nullptr) strm->bzfree = dflt_free;
  void* mem = strm->bzalloc(strm->opaque, (int)sizeof(DState), 1);
  if (mem == nullptr) return BZ_MEM_ERROR;
  DState* s = new (mem) DState();
  s->strm = strm;
  s->verbosity = verbosity;
  s->small = small;
  s->ph = kMagic;
  s->bb = 0;
  s->bl = 0;
  s->comb_crc = 0;
  s->out_pos = 0;
  s->stream_end_pending = false;
  strm->state = s;
  strm->total_in_lo32 = strm->total_in_hi32 = 0;
  strm->total_out_lo32 = strm->total_out_hi32 = 0;
  return BZ_OK;
}

int BZ2_bzDecompress(bz_stream* strm) {
  if (strm == nullptr || strm->state == nullptr) return BZ_PARAM_ERROR;
  DState* s = (DState*)strm->state;
  if (s->strm != strm) return BZ_PARAM_ERROR;
  if (s->ph == kError) return BZ_DATA_ERROR;
  for (;;) {
    drain(s);
    if (s->out_pos < s->out.size()) return BZ_OK;  // caller's output buffer is full
    if (s->stream_end_pending) return BZ_STREAM_END;
    if (s->ph == kDone) return BZ_SEQUENCE_ERROR;
    const Phase before = s->ph;
    const size_t out_before = s->out.size();
    int rc;
    try {
      rc = advance(s);
    } catch (const std::bad_alloc&) {
      return BZ_MEM_ERROR;
    }
    if (rc != BZ_OK) {
      s->ph = kError;
      return rc;
    }
    if (s->out.size() == out_before && !s->stream_end_pending && s->ph == before) return BZ_OK;  // needs input
  }
}

int BZ2_bzDecompressEnd(bz_stream* strm) {
  if (strm == nullptr || strm->state == nullptr) return BZ_PARAM_ERROR;
  DState* s = (DState*)strm->state;
  if (s->strm != strm) return BZ_PARAM_ERROR;
  s->~DState();
  strm->bzfree(strm->opaque, s);
  strm->state = nullptr;
  return BZ_OK;
}

}  // extern "C"
