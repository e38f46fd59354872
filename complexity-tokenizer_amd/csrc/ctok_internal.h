// Internal interfaces between the C++ host runtime (ctok_host.cpp) and the HIP kernels
// (kernels.hip).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ctok_dev {

// Merge table entry (u64): bits [0,21) = right id, [21,42) = left id, [42,64) = rank.
// Token ids must be < 2^21 - 1; ranks < 2^22 - 2.  All-ones = empty slot.
constexpr uint64_t kEmpty = ~0ull;
constexpr uint32_t kIdBits = 21;
constexpr uint64_t kKeyMask = (1ull << 42) - 1;
constexpr uint32_t kNoRank = 0x3FFFFFu;      // "no merge" (22-bit all ones)
constexpr uint32_t kMaxId = (1u << kIdBits) - 2;
constexpr uint32_t kPanicVal = kNoRank - 1;  // compact-table value of an entry whose lookup panics

// Error bits written by kernels into Workspace::err (host checks after the call).
constexpr uint32_t kErrPanic = 1u;

constexpr int kTile = 4096;        // bytes per pre-tokenizer tile
constexpr int kSegThreads = 256;   // 16 bytes per thread
constexpr int kHalo = 16;
constexpr int kShortMax = 32;      // pieces up to this many bytes are merged thread-per-piece

// Whole-piece table: raw byte strings of <= 8 bytes whose BPE is exactly one token (checked at
// load time by running the merge loop on every vocab entry).  Entry = {lo32, hi32, len, id} of
// the zero-padded bytes; len == 0 marks an empty slot.
__host__ __device__ inline uint32_t piece_hash(uint32_t lo, uint32_t hi, uint32_t len) {
  uint32_t h = lo * 0x9E3779B1u ^ (hi + 0x632BE5ABu) * 0x85EBCA77u ^ len * 0xC2B2AE3Du;
  return h ^ (h >> 16);
}

struct Tables {            // device pointers, owned by the host runtime
  const uint64_t* merge_tab;
  uint32_t merge_mask;     // capacity - 1 (power of two)
  const uint4* piece_tab;  // whole-piece table (see piece_hash)
  uint32_t piece_mask;
  const uint32_t* rank_newid;
  uint32_t n_ranks;
  const int32_t* byte2id;  // [256], -1 = byte char missing from vocab (dropped)
  const uint8_t* cls_s1;   // class two-level table (see gen/unicode_data.h)
  const uint8_t* cls_s2;
  const uint8_t* nfc_s1;
  const uint16_t* nfc_s2;
  const uint32_t* decomp_cp;
  const uint16_t* decomp_off;
  const uint32_t* decomp_data;
  uint32_t n_decomp;
  const uint64_t* comp_key;
  const uint32_t* comp_val;
  uint32_t n_comp;
  const uint8_t* bytemap_alnum;  // [256]
  // added tokens that can occur inside a piece (raw-byte patterns), usually none
  const uint8_t* at_bytes;
  const uint32_t* at_off;  // [n_at + 1]
  const uint32_t* at_id;
  const uint8_t* at_flags;  // bit0 single_word, bit1 lstrip, bit2 rstrip
  uint32_t n_at;
  uint32_t proper;          // 1: merge table is rank-monotone (parallel same-rank rounds exact)
  uint32_t compact;         // 1: entry values are new ids (strictly increasing in rank), else ranks
  uint32_t dbg;             // debug mode (CTOK_DBG_MODE), 0 in production
};

struct Work {              // device pointers, sized by the host for one call
  const uint8_t* text;     // (normalised) text
  uint32_t n_bytes;
  const uint64_t* doc_off; // (normalised) offsets, n_docs + 1
  uint32_t n_docs;
  uint32_t* docbits;       // doc-start bitmap, n_words + 2
  uint32_t* pbits;         // piece-start bitmap
  uint32_t n_words;
  uint32_t* tile_cnt;      // n_tiles + 1 (exclusive-scanned in place into tile_base)
  uint32_t n_tiles;
  uint32_t* word_prefix;   // n_words
  uint32_t* pstart;        // n_bytes + 1
  uint32_t* pcnt;          // n_bytes + 1 (scanned into ptok in place)
  uint32_t* scratch;       // n_bytes: tokens of piece p at scratch[pstart[p]..]
  uint32_t* doc_piece;     // n_docs + 1
  uint32_t* long_list;     // n_bytes / kShortMax + 1
  uint32_t* mid_list;      // pieces for the generic thread-per-piece kernel
  uint32_t* region;        // per routing block: class-0 pieces from the front, class 1 from the back
  uint32_t* region2;       // per routing block: class-2 pieces
  uint32_t region_len;     // entries per block (>= pieces per block)
  uint32_t grid1;          // blocks of the routing pass
  uint32_t* ccnt;          // [3][grid1 + 1] pieces per block and class, scanned to offsets
  uint32_t* dense;         // the three class lists gathered densely (k_compact)
  uint32_t* counters;      // [0] long count, [2] err, [3] nfc docs, [4] mid count, [5] list16 count
  uint32_t* lw;            // long-piece workspace: 4 * n_bytes u32
  uint32_t* scan_tmp;      // scan partials
  uint64_t scan_tmp_cap;
};

// ---- launchers (kernels.hip) -----------------------------------------------------------
void upload_done();
hipError_t launch_docstart(const Work& w, hipStream_t s);
hipError_t launch_nfc_check(const uint8_t* text, uint64_t n_bytes, const uint64_t* doc_off, uint32_t n_docs,
                            const Tables& t, uint32_t* doc_flag, uint32_t* counter, hipStream_t s);
hipError_t launch_norm(const uint8_t* text, const uint64_t* doc_off, uint32_t n_docs, const uint32_t* doc_flag,
                       int add_prefix, int nfc, const Tables& t, uint32_t* cp_scratch, uint32_t* ncp,
                       uint64_t* new_len_then_off, uint8_t* out_text, int phase, hipStream_t s);
hipError_t launch_segment(const Work& w, const Tables& t, hipStream_t s);
hipError_t launch_pieces(const Work& w, hipStream_t s);
hipError_t launch_bpe(const Work& w, const Tables& t, hipStream_t s);
hipError_t launch_bpe_long(const Work& w, const Tables& t, hipStream_t s);
hipError_t launch_emit(const Work& w, uint32_t* ids, uint64_t ids_cap, uint64_t* tok_off, hipStream_t s);
// exclusive scan of n u32 (n read from *n_dev when non-null, else n_max); out[n] = total
hipError_t scan_u32(const uint32_t* in, uint32_t* out, uint64_t n_max, const uint32_t* n_dev,
                    uint32_t* tmp, uint64_t tmp_cap, hipStream_t s);
hipError_t scan_u64(uint64_t* inout, uint64_t n, uint64_t* tmp, uint64_t tmp_cap, hipStream_t s);
uint64_t scan_tmp_elems(uint64_t n_max);

}  // namespace ctok_dev
