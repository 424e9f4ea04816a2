// stages.h -- the per-batch pipeline stages of the MI355X bzip2 engine and their shared
// device workspace.  A "batch" is a contiguous run of input bytes in HBM whose blocks are
// compressed together: RLE1/segmentation (rle1.hip) -> cyclic suffix sort and BWT
// (sort.hip) -> MTF/RUNA-RUNB (mtf.hip) -> table optimisation, Huffman codes and bit
// packing (code.hip).
#pragma once
#include <exception>
#include <functional>
#include <initializer_list>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace bzg {

// Device buffers keyed by name, grown on demand (contents are not preserved on growth).
class Workspace {
 public:
  Workspace() = default;
  ~Workspace();
  Workspace(const Workspace&) = delete;
  Workspace& operator=(const Workspace&) = delete;

  void* get(const std::string& name, size_t bytes, bool zero = false);
  uint8_t* u8(const std::string& name, size_t n) { return (uint8_t*)get(name, n); }
  uint16_t* u16(const std::string& name, size_t n) { return (uint16_t*)get(name, n * 2); }
  uint32_t* u32(const std::string& name, size_t n) { return (uint32_t*)get(name, n * 4); }
  // the same, zeroed (on this workspace's stream) whenever it is (re)allocated: scan scratch
  uint32_t* u32z(const std::string& name, size_t n) { return (uint32_t*)get(name, n * 4, true); }
  template <typename T>
  T* typed(const std::string& name, size_t n) { return (T*)get(name, n * sizeof(T)); }

  // Grow-only pinned host buffer, kept across calls (growth first waits for the side stream,
  // the only user of these buffers), and the workspace's side stream and events, created once.
  void* pinned(const std::string& name, size_t bytes);
  hipStream_t side_stream();
  hipEvent_t side_event(int k);  // k < 4: 0, 1 the A5 copy-rank job, 2, 3 the table streams' fork / join

  const uint32_t* crc_table();   // 256 entries, MSB-first CRC-32 (poly 0x04C11DB7)
  const uint32_t* xpow2_table(); // 48 entries: x^(8*2^k) mod P
  size_t bytes_reserved() const { return total_; }
  void release_all();
  // The stream that uses the workspace from now on: growth frees and allocates in that
  // stream's order (hipFreeAsync / hipMallocAsync) instead of synchronising the device, so
  // concurrent engines on one device never wait for each other.  A switch makes the new
  // stream wait for the work queued so far on the old one, so a later free on the new stream
  // is ordered after every earlier use of the buffers.
  void set_stream(hipStream_t s);
  // Copies `bytes` (4-byte aligned, small: the sort's list sizes between passes) from device
  // memory to `dst` once the work queued on `st` so far is done.  A one-workgroup kernel
  // writes them into pinned host memory and raises a flag there that this thread spins on: no
  // copy-engine transfer and no sleeping wait, so the device idles a few microseconds per
  // read instead of ~35 (profiles/r05_gaps_*).  Larger reads take hipMemcpyAsync + a stream
  // synchronisation.
  void read_small(void* dst, const void* dev_src, size_t bytes, hipStream_t st);
  // the same for up to four pieces at once; a piece with stride s > 1 reads the 32-bit words
  // src[0], src[s], src[2 s], ... (bytes / 4 of them)
  struct SmallRead {
    void* dst;
    const void* src;
    size_t bytes;
    uint32_t stride = 1;
  };
  void read_small(std::initializer_list<SmallRead> reads, hipStream_t st);

 private:
  struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    bool async = false;
  };
  void drop(Buf& b);
  hipStream_t stream_ = nullptr;
  hipEvent_t handoff_ = nullptr;
  std::map<std::string, Buf> bufs_;
  std::map<std::string, std::pair<void*, size_t>> pins_;
  hipStream_t side_ = nullptr;
  hipEvent_t sev_[4] = {};
  size_t total_ = 0;
  uint32_t* crc_ = nullptr;
  uint32_t* xp2_ = nullptr;
  uint32_t* mbox_ = nullptr;  // pinned host words for read_small, the flag after them
  uint32_t* mbox_dev_ = nullptr;
  uint32_t mseq_ = 0;
};

// ---- stage A1/A2 ---------------------------------------------------------------------
struct Rle1Result {
  uint64_t consumed = 0;  // input bytes covered by the emitted blocks
  uint32_t m = 0;         // RLE1 output bytes produced for the whole batch
  uint32_t nblocks = 0;
  // device arrays (owned by the workspace)
  uint8_t* blk = nullptr;       // block bytes, block b at [boff[b], boff[b+1])
  uint32_t* boff = nullptr;     // nblocks+1
  uint32_t* binst = nullptr;    // nblocks+1 input offsets (relative to batch start)
  uint32_t* bcrc = nullptr;     // finalised block CRC
  uint32_t* inuse = nullptr;    // 8 words per block
  uint32_t* ninuse = nullptr;
  uint32_t* period = nullptr;   // primitive period of each block
  uint32_t* bq = nullptr;       // B* offsets of each periodic block's root (origptr.hip)
  uint32_t* qper = nullptr;     // smallest period of a quasi-periodic block (qsa.h), else 0
};
// crc_st / crc_in / crc_out (optional): the block CRCs and the in-use maps run on crc_st, which
// waits for crc_in (recorded on st once their inputs are ready); crc_out is recorded after them,
// and bcrc / inuse / ninuse may be read only by work ordered after it (the sort reads neither).
void rle1_stage(Workspace& ws, const uint8_t* d_in, uint64_t n, int level, bool final_batch,
                bool tail_merge, Rle1Result& res, hipStream_t st, hipStream_t crc_st = nullptr,
                hipEvent_t crc_in = nullptr, hipEvent_t crc_out = nullptr);
// in-use maps, nInUse and primitive periods of res.nblocks blocks given res.blk / res.boff
// (side: the in-use maps go there; only MTF and the tables read them)
void block_info_stage(Workspace& ws, Rle1Result& res, hipStream_t st, hipStream_t side = nullptr);
// bit offsets of the block-header / end-of-stream magics of a .bz2 stream, sorted, as
// 2 * offset + kind (magic.hip)
uint64_t find_magics_stage(const uint8_t* d_in, uint64_t n, std::vector<uint64_t>& found, hipStream_t st);
// one region of a sharded stream: RLE1 chunk map, then block cuts for a given
// open-block fill at the region start (input offsets relative to the region)
void seg_map_stage(Workspace& ws, const uint8_t* d_in, uint64_t n, hipStream_t st);
void seg_walk_stage(Workspace& ws, const uint8_t* d_in, uint64_t n, int level, uint32_t fill_in,
                    bool final_region, std::vector<uint64_t>& cuts, uint64_t& last_chunk, uint32_t& last_fill,
                    hipStream_t st);

// ---- stage A5 (origptr.hip) ----------------------------------------------------------
// B* offsets per periodic root (part of block_info_stage); the copy ranks of the roots with
// more than one (origptr.hip: the device's closed form, then the host model for the rest on a
// side stream, started before the sort and overlapping it); origptr after the sort.
struct CopyRankJob {
  std::vector<uint32_t> need, per, len;  // blocks with such roots, their periods and lengths
  int32_t* dev_r = nullptr;              // per block: r (workspace buffer)
  // the part workspace's pinned buffers, side stream and events (reused from batch to batch)
  int32_t* pin_r = nullptr;              // pinned: the device's answers, then the merged ones
  uint8_t* pin_roots = nullptr;          // pinned: the roots of `need`, concatenated
  hipStream_t side = nullptr;
  hipEvent_t ev_cf = nullptr, ev_done = nullptr;
  uint32_t n_host = 0;  // roots the host model resolved
  int failed = 0;
  CopyRankJob() = default;
  CopyRankJob(const CopyRankJob&) = delete;
  CopyRankJob& operator=(const CopyRankJob&) = delete;
  ~CopyRankJob();
};
void copyrank_count_stage(Rle1Result& r, Workspace& ws, hipStream_t st);
void copyrank_memo_clear();  // bzg_release: drops the memoised periodic roots
void copyrank_begin(Workspace& ws, const Rle1Result& r, const std::vector<uint32_t>& hboff,
                    const std::vector<uint32_t>& hper, const std::vector<uint32_t>& hbq, CopyRankJob& job,
                    hipStream_t st);
void copyrank_finish(Workspace& ws, const Rle1Result& r, const uint32_t* rank0, uint32_t* origptr, CopyRankJob& job,
                     hipStream_t st);
// after the batch's last synchronisation: throws if the host model failed on a root
void copyrank_check(const CopyRankJob& job);

// ---- stage A4 ------------------------------------------------------------------------
// Sorts the rotations of every block (of its primitive root when periodic) and writes the
// BWT last column to `bwt` (same offsets as the blocks) and rank0[b] = rank of rotation 0
// among the distinct rotations of the root.
struct SortStats {
  int iterations = 0;
  uint64_t unsorted_elems = 0;  // sum over iterations of elements in unsorted groups
  int s2_iters = 0;             // S2 rounds of run emission
};
// h_qper (optional): r.qper on the host; those blocks are ordered analytically (qsa.h).
void bwt_stage(Workspace& ws, const Rle1Result& r, const std::vector<uint32_t>& h_boff,
               const std::vector<uint32_t>& h_period, uint8_t* bwt, uint32_t* rank0,
               SortStats* stats, hipStream_t st, const uint32_t* h_qper = nullptr);

// ---- stage A6 ------------------------------------------------------------------------
struct MtfResult {
  uint16_t* mtfv = nullptr;   // block b at [mtf_off[b], mtf_off[b] + nmtf[b])
  uint32_t* mtf_off = nullptr;
  uint32_t* nmtf = nullptr;
  uint32_t* freq = nullptr;   // 258 per block
};
void mtf_stage(Workspace& ws, const Rle1Result& r, const uint8_t* bwt, uint32_t nblocks,
               uint32_t total_bytes, MtfResult& res, hipStream_t st, const std::vector<uint32_t>* host_boff = nullptr);

// ---- stage A7/A8/A3 --------------------------------------------------------------------
struct StreamCarry {
  uint32_t combined_crc = 0;
  uint8_t carry_byte = 0;   // pending high bits of an unfinished output byte
  uint8_t carry_bits = 0;   // 0..7
  bool header_done = false;
};
// Encodes all blocks into `out` (device), starting with the carried partial byte; when
// `final_batch` appends the stream trailer.  Returns bytes fully written; updates carry.
// Test hook: BZ2_hbMakeCodeLengths on n tables (kMaxAlpha frequencies each) on the GPU.
void code_lengths_test(Workspace& ws, const uint32_t* d_freq, const int32_t* d_alpha, uint32_t n, int max_len,
                       uint8_t* d_lens, hipStream_t st);
// The per-block tables of nb blocks (selectors, code lengths, canonical codes, bit counts).
struct CodeTables {
  uint8_t* lens = nullptr;
  uint32_t* codes = nullptr;
  uint8_t* sel = nullptr;
  uint8_t* selmtf = nullptr;
  uint16_t* gbits = nullptr;
  uint32_t* info = nullptr;
  uint64_t* bbits = nullptr;
};
void code_tables(Workspace& ws, const Rle1Result& r, const MtfResult& m, uint32_t nb, CodeTables& t, hipStream_t st,
                 hipStream_t st2 = nullptr);
// One part of a batch (consecutive blocks, in stream order) ready to be packed.
struct CodePart {
  const Rle1Result* r;
  const MtfResult* m;
  const CodeTables* t;
  const uint32_t* origptr;
  uint32_t nb;
};
// Bit offsets across the parts, then the packed stream (header / trailer as needed).
uint64_t code_emit(Workspace& ws, const std::vector<CodePart>& parts, int level, bool final_batch, StreamCarry& carry,
                   uint8_t* out, uint64_t out_cap, hipStream_t st);
uint64_t code_stage(Workspace& ws, const Rle1Result& r, const MtfResult& m, const uint32_t* origptr,
                    uint32_t nblocks, int level, bool final_batch, StreamCarry& carry, uint8_t* out,
                    uint64_t out_cap, hipStream_t st);

// ---- decompression (decomp.hip) --------------------------------------
struct DecodeStats {
  uint64_t candidates = 0;  // block magics decoded (real blocks + chance matches)
  uint64_t blocks = 0;
  uint64_t out_bytes = 0;
  float total_ms = 0;
};
// Decodes the .bz2 stream d_in[0, n) into d_out[0, out_cap).  Returns BZ_OK for a complete,
// correct stream, else the code BZ2_bzBuffToBuffDecompress returns (bzlib.c:1361-1410);
// *out_len = bytes written.
int decode_stage(Workspace& ws, const uint8_t* d_in, uint64_t n, uint8_t* d_out, uint64_t out_cap,
                 uint64_t* out_len, DecodeStats* stats, hipStream_t st);

}  // namespace bzg
